#!/bin/bash
# Collect one round's measurement artifacts on the GPU box (run from the repo root via gpurun):
#   tools/profile_round.sh <tag> [bench args]   e.g.  tools/profile_round.sh r01 ; ... r01_r50 --workload resnet50
# -> gpurun_out/prof_<tag>/: bench.json (default bench: roofline + cpu_baseline), kernel-trace
#    stats of the graph-replayed step, and FETCH_SIZE / WRITE_SIZE passes (separate, as the
#    MI355X guide prescribes; eager mode) summarised into pmc_traffic.json.
set -euo pipefail
TAG=${1:?tag}
shift
EXTRA="$*"  # extra bench.py arguments, e.g. --workload resnet50
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_$TAG
rm -rf "$OUT" && mkdir -p "$OUT"
timeout -k 10 400 python bench.py $EXTRA > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
  python bench.py $EXTRA --steps 50 --warmup 10 --no-cpu-baseline --no-roofline > "$OUT/stats.log" 2>&1
echo "stats done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python bench.py $EXTRA --steps 3 --warmup 1 --eager --no-cpu-baseline --no-roofline > "$OUT/fetch.log" 2>&1
echo "fetch done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python bench.py $EXTRA --steps 3 --warmup 1 --eager --no-cpu-baseline --no-roofline > "$OUT/write.log" 2>&1
echo "write done"
python tools/pmc_summary.py "$OUT/fetch" "$OUT/write" "$OUT/pmc_traffic.json" > /dev/null

timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_VALU_MFMA_MOPS_F16 \
  --output-format csv -d "$OUT/mfma" -o run -- \
  python bench.py $EXTRA --steps 3 --warmup 1 --eager --no-cpu-baseline --no-roofline > "$OUT/mfma.log" 2>&1
python tools/mfma_summary.py "$OUT/mfma" "$OUT/mfma_util.json" > /dev/null
echo "mfma done"
echo "all done"
