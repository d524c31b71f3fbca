#!/bin/bash
# Interleaved A/B of environment switches on the GPU box: tools/ab_env.sh OUT ROUNDS "ENV_A" "ENV_B" [...]
#   [-- bench args]
# e.g. tools/ab_env.sh gpurun_out/x 3 "LBT_HEAD_CHAIN=1" "LBT_HEAD_CHAIN=0". Default bench, 300 steps.
set -uo pipefail
OUT=$1; ROUNDS=$2; shift 2
ENVS=(); ARGS=(--steps 300 --warmup 30)
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; ARGS=("$@"); break; fi
  ENVS+=("$1"); shift
done
set -- "${ENVS[@]}"
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for E in "$@"; do
    i=$((i + 1))
    env $E timeout -k 10 300 python bench.py "${ARGS[@]}" --no-cpu-baseline --no-roofline \
      > "$OUT/v${i}_$r.json" 2> "$OUT/v${i}_$r.err" || { echo "bench [$E] failed"; exit 1; }
    echo "[$E] round $r: $(python -c "import json;d=json.load(open('$OUT/v${i}_$r.json'));print(d['ms_per_step'], d['value'])")"
  done
done
