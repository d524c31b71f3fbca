#!/bin/bash
# Diagnostics of igemm_big_kernel on the GPU box: ring depth (LBT_IGEMM_BIG_S), loads switched off
# after the prologue (LBT_IGEMM_BIG_DBG=1: the MFMA + LDS-read bound), and SQ counters on two shapes.
# -> gpurun_out/igdiag/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/igdiag; mkdir -p $OUT
for v in ${IGDIAG_VARIANTS:-"S4:LBT_IGEMM_BIG_S=4" "S3:LBT_IGEMM_BIG_S=3" "S2:LBT_IGEMM_BIG_S=2" "old:LBT_IGEMM_BIG=0"}; do
  tag=${v%%:*}; envs=${v#*:}
  env ${envs//,/ } timeout -k 10 120 python tools/igemm_probe.py > $OUT/probe_$tag.txt 2>&1 || exit 1
  echo "== $tag"; grep -v amdgpu $OUT/probe_$tag.txt | cut -c1-60
done
[ -n "${IGDIAG_PMC:-}" ] || { echo done; exit 0; }
export PROBE_ONLY=$IGDIAG_PMC
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc1 -o run -- \
  python tools/igemm_probe.py > $OUT/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc2 -o run -- \
  python tools/igemm_probe.py > $OUT/pmc2.log 2>&1 || exit 1
echo done
