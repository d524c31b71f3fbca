set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
CHECK_DP=1 bash tools/gpu_check.sh r04v || exit 1
mkdir -p gpurun_out/r04v
timeout -k 10 400 python bench.py --workload resnet50 --steps 20 --warmup 5 > gpurun_out/r04v/resnet50_bench.json 2> gpurun_out/r04v/resnet50_bench.err; rc=$?
cat gpurun_out/r04v/resnet50_bench.json; [ $rc = 0 ] || exit 1
timeout -k 10 300 python bench.py --workload resnet20w4 > gpurun_out/r04v/resnet20w4_bench.json 2> gpurun_out/r04v/resnet20w4_bench.err; rc=$?
cat gpurun_out/r04v/resnet20w4_bench.json
echo done
