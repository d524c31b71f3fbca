#!/bin/bash
# A/B of library builds on the GPU box: tools/ab_run.sh OUT FILTER LIB1 [LIB2 ...]
# per-launch graph-replay times (tools/launch_bench.py --filter FILTER) and a short bench per build.
set -uo pipefail
OUT=$1; FILTER=$2; shift 2
mkdir -p "$OUT"
for L in "$@"; do
  T=$(basename "$(dirname "$L")"); [ "$T" = lbt_amd ] && T=main
  L=$(realpath "$L")
  LBT_LIBRARY=$L timeout -k 10 120 python tools/launch_bench.py --filter "$FILTER" > "$OUT/lb_$T.log" 2>&1 || { echo "launch_bench $T failed"; exit 1; }
  LBT_LIBRARY=$L timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-roofline > "$OUT/bench_$T.json" 2> "$OUT/bench_$T.err" || { echo "bench $T failed"; exit 1; }
  echo "$T: $(python -c "import json;d=json.load(open('$OUT/bench_$T.json'));print(d['ms_per_step'], d['value'])")"
done
