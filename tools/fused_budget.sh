#!/bin/bash
# Per-phase budget of the fused ResNet-20 conv kernels: per-workgroup phase
# timestamps of every conv_bwd_kernel / conv_fwd_fused_kernel launch of the step (isolated graph replay,
# warm and with the caches flushed first), the load phase split (-DLBT_P1STUDY build), and one SQ
# counter pass over two eager B=128 steps restricted to those kernels (VALU instructions per element).
#   tools/fused_budget.sh <tag>     (run from the repo root via gpurun; the trace builds are made here
#   first: python tools/trace_phases.py --build; python tools/build_variant.py p1study -DLBT_TRACE -DLBT_P1STUDY)
set -uo pipefail
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for K in conv_bwd_kernel conv_fwd_fused_kernel; do
  for mode in warm cold; do
    extra=""; [ $mode = cold ] && extra="--cold"
    timeout -k 10 200 python tools/trace_phases.py --filter $K $extra > "$OUT/trace_${K}_$mode.txt" 2>&1 \
      || { echo "trace $K $mode failed"; exit 1; }
    echo "trace $K $mode done"
  done
  timeout -k 10 200 python tools/trace_phases.py --filter $K --cold --lib lbt_amd/build_var/p1study/liblbt_dfxp.so \
    > "$OUT/trace_${K}_p1study_cold.txt" 2>&1 || { echo "p1study $K failed"; exit 1; }
done
RX='conv_bwd_kernel|conv_fwd_fused_kernel'
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-include-regex "$RX" --output-format csv -d "$OUT/sq" -o run -- \
  python bench.py --steps 2 --warmup 1 --eager --no-cpu-baseline --no-roofline > "$OUT/sq.log" 2>&1 \
  || { echo "sq pass failed"; exit 1; }
python tools/sq_summary.py "$OUT/sq" > "$OUT/sq_summary.txt" 2>&1 || true
python tools/pmc_dump.py "$OUT/sq" > "$OUT/sq_dump.txt" 2>&1 || true
echo done
