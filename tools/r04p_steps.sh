set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04p
timeout -k 10 300 python -u -m pytest tests/test_igemm_big.py -m gpu -v --timeout 240 -k "bna or bn3 or fwd or quantising" \
  --timeout-method thread > gpurun_out/r04p/first.log 2>&1; rc=$?
tail -3 gpurun_out/r04p/first.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python tools/bna_probe.py > gpurun_out/r04p/bna_probe.txt 2>&1; rc=$?
cat gpurun_out/r04p/bna_probe.txt; [ $rc = 0 ] || exit 1
S3=l1_c2_fwd,l2_c2_fwd,l3_c2_fwd,l4_c2_fwd,l1_c2_fwdq,l2_c2_fwdq,l3_c2_fwdq
for h in 1 0; do
  LBT_IGEMM_HALO=$h PROBE_ONLY=$S3 PROBE_QNOISE=table timeout -k 10 240 python tools/igemm_probe.py \
    > gpurun_out/r04p/probe_halo$h.txt 2>&1 || { echo "probe failed"; tail -3 gpurun_out/r04p/probe_halo$h.txt; exit 1; }
  echo "== halo $h"; cat gpurun_out/r04p/probe_halo$h.txt
done
bash tools/ab_env.sh gpurun_out/r04p_r50 2 "LBT_IGEMM_HALO=1" "LBT_IGEMM_HALO=1 LBT_DGRAD_BN3_PY=0" "LBT_IGEMM_HALO=1 LBT_DGRAD_BNA_PY=0 LBT_DGRAD_BN3_PY=0" "LBT_IGEMM_HALO=0 LBT_DGRAD_BNA_PY=0 LBT_DGRAD_BN3_PY=0" -- --workload resnet50 --steps 20 --warmup 5 || exit 1
echo done
