set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r50
timeout -k 10 300 python bench.py --workload resnet50 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/r50/b32.json 2> gpurun_out/r50/b32.err && echo b32 ok
timeout -k 10 300 python bench.py --workload resnet50 --batch 128 --steps 6 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/r50/b128.json 2> gpurun_out/r50/b128.err && echo b128 ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r50/stats -o run -- python bench.py --workload resnet50 --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/r50/stats.log 2>&1 && echo stats ok
