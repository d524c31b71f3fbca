#!/bin/bash
# Counter breakdown of the ResNet-50 element chains (forward chain, pass B): per-launch algorithmic
# bandwidth (tools/kernel_bw.py --detail) and three rocprofv3 --pmc passes over eager steps restricted to
# those kernels (PMC slots: SQ 8, TCC 4, GRBM 2; each pass its own run under a KILL time limit).
#   tools/chain_pmc.sh <tag>      -> gpurun_out/<tag>/  (run from the repo root via gpurun)
set -uo pipefail
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 300 python tools/kernel_bw.py --workload resnet50 --detail chain_fwd_kernel bn_bwd_b_wide_kernel \
  > "$OUT/kernel_bw.txt" 2>&1 || { echo "kernel_bw failed"; exit 1; }
echo "kernel_bw done"
RX='chain_fwd_kernel|bn_bwd_b_wide_kernel'
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc$i" -o run -- \
    python bench.py --workload resnet50 --steps 2 --warmup 1 --eager --no-cpu-baseline --no-roofline \
    > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
  echo "pmc pass $i done"
done
python tools/pmc_dump.py "$OUT" > "$OUT/summary.txt" 2>&1 || true
echo done
