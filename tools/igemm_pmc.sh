#!/bin/bash
# Counter breakdown of the two worst ResNet-50 GEMMs: l1_c2 3x3 fwdq and l1_c3 1x1
# fwdq, with their fp32-output twins (the epilogue's share = fwdq - fwd) and the three noise sources of
# the quantising epilogue (Philox inline, per-step table, none = round-to-nearest).
#   tools/igemm_pmc.sh <tag>      -> gpurun_out/<tag>/  (run from the repo root via gpurun)
# Each rocprofv3 pass is its own run under a KILL time limit (PMC slots: SQ 8, TCC 4, GRBM 2).
set -uo pipefail
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
SHAPES=${IGPMC_SHAPES:-l1_c2_fwdq,l1_c2_fwd,l1_c3_fwdq,l1_c3_fwd}
for qn in inline table none; do
  PROBE_ONLY=$SHAPES PROBE_QNOISE=$qn timeout -k 10 120 python tools/igemm_probe.py > "$OUT/probe_$qn.txt" 2>&1 || exit 1
  echo "== noise $qn"; grep -v amdgpu "$OUT/probe_$qn.txt" | cut -c1-100
done
export PROBE_QNOISE=table PROBE_ONLY=$SHAPES
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_WAVES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc$i" -o run -- \
    python tools/igemm_probe.py > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
  echo "pmc pass $i done"
done
python tools/sq_summary.py "$OUT" > "$OUT/summary.txt" 2>&1 || true
echo done
