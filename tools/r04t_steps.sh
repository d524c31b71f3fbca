set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04t
timeout -k 10 400 python -u -m pytest tests/test_igemm_big.py tests/test_resnet50.py -m gpu -v --timeout 240 \
  --timeout-method thread > gpurun_out/r04t/first.log 2>&1; rc=$?
tail -3 gpurun_out/r04t/first.log; [ $rc = 0 ] || exit 1
S=l1_c2_fwdq,l2_c2_fwdq,l3_c2_fwdq,l1_c3_fwdq,l3_c3_fwdq
for v in 1 0; do
  LBT_FWDQ_PERM=$v PROBE_ONLY=$S PROBE_QNOISE=table timeout -k 10 240 python tools/igemm_probe.py \
    > gpurun_out/r04t/probe_perm$v.txt 2>&1 || { echo "probe failed"; tail -3 gpurun_out/r04t/probe_perm$v.txt; exit 1; }
  echo "== fwdq_perm $v"; cat gpurun_out/r04t/probe_perm$v.txt
done
bash tools/ab_env.sh gpurun_out/r04t_r50 2 "LBT_FWDQ_PERM=1" "LBT_FWDQ_PERM=0" -- --workload resnet50 --steps 20 --warmup 5 || exit 1
echo done
