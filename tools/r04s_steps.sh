set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04s
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04s/prof -o run -- python bench.py --workload resnet50 --steps 10 --warmup 3 --no-roofline --no-cpu-baseline > gpurun_out/r04s/bench.json 2> gpurun_out/r04s/bench.err; rc=$?
cat gpurun_out/r04s/bench.json; [ $rc = 0 ] || exit 1
echo done
