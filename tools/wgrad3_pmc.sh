#!/bin/bash
# SQ counters of the all-taps 3x3 wgrad on the l1_c2 / l3_c2 shapes -> gpurun_out/w3pmc/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/w3pmc; mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/p1 -o run -- \
  python tools/wgrad3_probe.py > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_I8 \
  --output-format csv -d $OUT/p2 -o run -- python tools/wgrad3_probe.py > $OUT/p2.log 2>&1 || exit 1
echo done
