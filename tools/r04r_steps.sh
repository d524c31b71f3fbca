set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04r
timeout -k 10 400 python -u -m pytest tests/test_igemm_big.py tests/test_resnet50.py -m gpu -v --timeout 240 \
  --timeout-method thread > gpurun_out/r04r/first.log 2>&1; rc=$?
tail -3 gpurun_out/r04r/first.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python tools/bna_probe.py > gpurun_out/r04r/bna_probe.txt 2>&1; rc=$?
cat gpurun_out/r04r/bna_probe.txt; [ $rc = 0 ] || exit 1
bash tools/ab_env.sh gpurun_out/r04r_r50 2 "LBT_IGEMM_HALO=1" "LBT_IGEMM_HALO=1 LBT_DGRAD_BN3_PY=0" "LBT_IGEMM_HALO=1 LBT_DGRAD_BNA_PY=0 LBT_DGRAD_BN3_PY=0" -- --workload resnet50 --steps 20 --warmup 5 || exit 1
echo done
