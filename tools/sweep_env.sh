#!/bin/bash
# A/B of environment settings on the GPU box: tools/sweep_env.sh OUT FILTER "ENV1" "ENV2" ...
# (each ENV a space-separated list of VAR=value); per-launch graph-replay times + a 300-step bench.
set -uo pipefail
OUT=$1; FILTER=$2; shift 2
mkdir -p "$OUT"
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 120 python tools/launch_bench.py --filter "$FILTER" > "$OUT/lb_$i.log" 2>&1 || { echo "lb $E failed"; exit 1; }
  env $E timeout -k 10 120 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-roofline > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || { echo "bench $E failed"; exit 1; }
  echo "[$E] $(grep -E "^ +[0-9]+ " "$OUT/lb_$i.log" | awk '{s+=$2} END{print s}') us | $(python -c "import json;d=json.load(open('$OUT/bench_$i.json'));print(d['ms_per_step'])") ms"
done
