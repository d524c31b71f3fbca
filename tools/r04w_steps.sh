set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04w
timeout -k 10 300 python -u -m pytest tests/test_edge_cases.py -m gpu -v --timeout 120 --timeout-method thread -k prepare > gpurun_out/r04w/prepare.log 2>&1; rc=$?
tail -2 gpurun_out/r04w/prepare.log; [ $rc = 0 ] || exit 1
LBT_DIST_BACKEND=gloo LBT_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/r04w/dp2_weak.json 2> gpurun_out/r04w/dp2_weak.err; rc=$?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04w/dp2_weak.json; [ $rc = 0 ] || exit 1
LBT_HEAD=9b78ab4 bash tools/profile_round.sh r04w || exit 1
LBT_HEAD=9b78ab4 bash tools/profile_round.sh r04w_r50 --workload resnet50 --steps 20 --warmup 5 || exit 1
echo done
