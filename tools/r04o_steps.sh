set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04o
timeout -k 10 500 python -u -m pytest tests/test_igemm_big.py tests/test_resnet50.py -m gpu -x -v --timeout 240 \
  --timeout-method thread > gpurun_out/r04o/first.log 2>&1; rc=$?
tail -3 gpurun_out/r04o/first.log; [ $rc = 0 ] || exit 1
CHECK_DP=0 bash tools/gpu_check.sh r04o || exit 1
bash tools/ab_env.sh gpurun_out/r04o_r50 2 "LBT_DGRAD_BNA_PY=1 LBT_DGRAD_BN3_PY=1" "LBT_DGRAD_BNA_PY=1 LBT_DGRAD_BN3_PY=0" "LBT_DGRAD_BNA_PY=0 LBT_DGRAD_BN3_PY=0" -- --workload resnet50 --steps 20 --warmup 5 || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04o_fetchcal -o run -- tools/fetch_cal > gpurun_out/r04o_fetchcal.log 2>&1
echo "done"
