set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05
timeout -k 10 300 python tools/stem_probe.py > gpurun_out/r05/stem_probe.txt 2>&1; rc=$?
cat gpurun_out/r05/stem_probe.txt; [ $rc = 0 ] || exit 1
CHECK_DP=1 bash tools/gpu_check.sh r05 || exit 1
timeout -k 10 400 python bench.py --workload resnet50 --steps 20 --warmup 5 > gpurun_out/r05/resnet50_bench.json 2> gpurun_out/r05/resnet50_bench.err; rc=$?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/resnet50_bench.json; [ $rc = 0 ] || exit 1
LBT_HEAD=02d6076 bash tools/profile_round.sh r05 || exit 1
LBT_HEAD=02d6076 bash tools/profile_round.sh r05_r50 --workload resnet50 --steps 20 --warmup 5 || exit 1
bash tools/ab_env.sh gpurun_out/r05_cg 1 "LBT_STEM_CG=32" "LBT_STEM_CG=64" -- --workload resnet50 --steps 20 --warmup 5 || exit 1
echo done
