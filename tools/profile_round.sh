#!/bin/bash
# Collect one round's measurement artifacts on the GPU box (run from the repo root via gpurun):
#   tools/profile_round.sh <tag>     e.g.  tools/profile_round.sh r01
# -> gpurun_out/prof_<tag>/: bench.json (default bench: roofline + cpu_baseline), kernel-trace
#    stats of the graph-replayed step, and FETCH_SIZE / WRITE_SIZE passes (separate, as the
#    MI355X guide prescribes; eager mode) summarised into pmc_traffic.json.
set -euo pipefail
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_$TAG
rm -rf "$OUT" && mkdir -p "$OUT"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
  python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-roofline > "$OUT/stats.log" 2>&1
echo "stats done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python bench.py --steps 3 --warmup 1 --eager --no-cpu-baseline --no-roofline > "$OUT/fetch.log" 2>&1
echo "fetch done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python bench.py --steps 3 --warmup 1 --eager --no-cpu-baseline --no-roofline > "$OUT/write.log" 2>&1
echo "write done"
python tools/pmc_summary.py "$OUT/fetch" "$OUT/write" "$OUT/pmc_traffic.json" > /dev/null
echo "all done"
