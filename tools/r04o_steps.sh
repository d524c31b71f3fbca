set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04o
timeout -k 10 500 python -u -m pytest tests/test_igemm_big.py tests/test_resnet50.py -m gpu -v --timeout 240 \
  --timeout-method thread > gpurun_out/r04o/first.log 2>&1; rc=$?
tail -3 gpurun_out/r04o/first.log; [ $rc = 0 ] || exit 1
S3=l1_c2_fwd,l2_c2_fwd,l3_c2_fwd,l4_c2_fwd,l1_c2_dgrad16,l2_c2_dgrad16,l3_c2_dgrad16,l4_c2_dgrad16,l1_c2_fwdq,l2_c2_fwdq,l3_c2_fwdq
for h in 1 0; do
  LBT_IGEMM_HALO=$h PROBE_ONLY=$S3 PROBE_QNOISE=table timeout -k 10 240 python tools/igemm_probe.py \
    > gpurun_out/r04o/probe_halo$h.txt 2>&1 || { echo "probe failed"; tail -3 gpurun_out/r04o/probe_halo$h.txt; exit 1; }
  echo "== halo $h"; cat gpurun_out/r04o/probe_halo$h.txt
done
CHECK_DP=0 bash tools/gpu_check.sh r04o || exit 1
bash tools/ab_env.sh gpurun_out/r04o_r50 2 "LBT_IGEMM_HALO=1" "LBT_IGEMM_HALO=0" "LBT_IGEMM_HALO=0 LBT_DGRAD_BNA_PY=0 LBT_DGRAD_BN3_PY=0" -- --workload resnet50 --steps 20 --warmup 5 || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04o_fetchcal -o run -- tools/fetch_cal > gpurun_out/r04o_fetchcal.log 2>&1
echo "done"
