#!/bin/bash
# Interleaved A/B of library builds on the GPU box: tools/ab_bench.sh OUT ROUNDS LIB1 LIB2 [...] [-- bench args]
# Each round runs the default bench (graph replay, 300 steps, no roofline / CPU baseline) once per build.
set -uo pipefail
OUT=$1; ROUNDS=$2; shift 2
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for L in "${LIBS[@]}"; do
    T=$(basename "$(dirname "$L")"); [ "$T" = lbt_amd ] && T=main
    LBT_LIBRARY=$(realpath "$L") timeout -k 10 180 python bench.py --steps 300 --warmup 30 --no-cpu-baseline \
      --no-roofline "$@" > "$OUT/${T}_$r.json" 2> "$OUT/${T}_$r.err" || { echo "bench $T failed"; exit 1; }
    echo "$T round $r: $(python -c "import json;d=json.load(open('$OUT/${T}_$r.json'));print(d['ms_per_step'], d['value'])")"
  done
done
