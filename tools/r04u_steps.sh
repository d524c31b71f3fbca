set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04u
timeout -k 10 400 python -u -m pytest tests/test_resnet50.py tests/test_igemm_big.py -m gpu -v --timeout 240 \
  --timeout-method thread > gpurun_out/r04u/first.log 2>&1; rc=$?
tail -3 gpurun_out/r04u/first.log; [ $rc = 0 ] || exit 1
for L in lbt_amd/liblbt_dfxp.so lbt_amd/build_var/u4/liblbt_dfxp.so lbt_amd/build_var/u8/liblbt_dfxp.so; do
  T=$(basename "$(dirname "$L")"); [ "$T" = lbt_amd ] && T=main
  LBT_LIBRARY=$(realpath "$L") timeout -k 10 300 python tools/bna_probe.py > gpurun_out/r04u/bna_$T.txt 2>&1 || { echo "bna probe $T failed"; exit 1; }
  LBT_LIBRARY=$(realpath "$L") PROBE_ONLY=l1_c2_fwdq,l2_c2_fwdq,l3_c2_fwdq,l1_c3_fwdq,l3_c3_fwdq PROBE_QNOISE=table \
    timeout -k 10 240 python tools/igemm_probe.py > gpurun_out/r04u/fwdq_$T.txt 2>&1 || { echo "probe $T failed"; exit 1; }
  echo "== $T"; cat gpurun_out/r04u/bna_$T.txt gpurun_out/r04u/fwdq_$T.txt
done
bash tools/ab_bench.sh gpurun_out/r04u_r50 2 lbt_amd/liblbt_dfxp.so lbt_amd/build_var/u4/liblbt_dfxp.so -- --workload resnet50 --steps 20 --warmup 5 || exit 1
echo done
