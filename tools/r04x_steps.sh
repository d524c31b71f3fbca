set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04x
timeout -k 10 400 python -u -m pytest tests/test_resnet50.py tests/test_igemm_big.py tests/test_dp_resnet50_gpu.py -m gpu -v --timeout 240 \
  --timeout-method thread > gpurun_out/r04x/first.log 2>&1; rc=$?
tail -3 gpurun_out/r04x/first.log; [ $rc = 0 ] || exit 1
bash tools/ab_env.sh gpurun_out/r04x_r50 2 "LBT_CHAIN_MS=1" "LBT_CHAIN_MS=0" -- --workload resnet50 --steps 20 --warmup 5 || exit 1
echo done
