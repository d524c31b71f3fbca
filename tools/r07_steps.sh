set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r07
for L in lbt_amd/liblbt_dfxp.so lbt_amd/build_var/q64/liblbt_dfxp.so; do
  T=$(basename "$(dirname "$L")"); [ "$T" = lbt_amd ] && T=main
  LBT_LIBRARY=$(realpath "$L") PROBE_ONLY=l1_c3_fwdq,l3_c3_fwdq PROBE_QNOISE=table timeout -k 10 240 python tools/igemm_probe.py > gpurun_out/r07/fwdq_$T.txt 2>&1 || { echo "probe $T failed"; exit 1; }
  echo "== $T"; cat gpurun_out/r07/fwdq_$T.txt
done
bash tools/ab_bench.sh gpurun_out/r07_r50 2 lbt_amd/liblbt_dfxp.so lbt_amd/build_var/pbu4/liblbt_dfxp.so lbt_amd/build_var/q64/liblbt_dfxp.so -- --workload resnet50 --steps 20 --warmup 5 || exit 1
echo done
