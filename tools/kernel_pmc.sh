#!/bin/bash
# SQ / LDS counter passes over two eager ResNet-20 steps for the kernels matching a regex (diagnostics):
#   tools/kernel_pmc.sh <tag> <kernel-regex> [bench args...]   -> gpurun_out/<tag>/pmc*/ + summary.txt
# Each pass is its own rocprofv3 run under a KILL time limit (SQ <= 8, GRBM <= 2, TCC <= 4 per pass).
set -uo pipefail
TAG=${1:?tag}; RX=${2:?regex}; shift 2
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_VMEM"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc$i" -o run -- \
    python bench.py --steps 2 --warmup 1 --eager --no-cpu-baseline --no-roofline "$@" > "$OUT/pmc$i.log" 2>&1 \
    || { echo "pmc pass $i failed"; tail -5 "$OUT/pmc$i.log"; continue; }
  echo "pmc pass $i done"
done
python tools/pmc_dump.py "$OUT" > "$OUT/summary.txt" 2>&1 || true
echo done
