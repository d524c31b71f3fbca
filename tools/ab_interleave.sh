#!/bin/bash
# Interleaved A/B of library builds on ONE GPU box (box-to-box spread is +-2 %, so only same-box,
# interleaved runs compare): tools/ab_interleave.sh OUT REPS LIB1 [LIB2 ...] [-- extra bench args]
# Each rep runs bench.py (200 timed steps) once per build, in turn; prints ms/step per build per rep.
set -uo pipefail
OUT=$1; REPS=$2; shift 2
LIBS=(); EXTRA=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; EXTRA=("$@"); break; fi
  LIBS+=("$1"); shift
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for L in "${LIBS[@]}"; do
    T=$(basename "$(dirname "$L")"); [ "$T" = lbt_amd ] && T=main
    L=$(realpath "$L")
    LBT_LIBRARY=$L timeout -k 10 150 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-roofline "${EXTRA[@]}" \
      > "$OUT/bench_${T}_$rep.json" 2> "$OUT/bench_${T}_$rep.err" || { echo "bench $T failed"; exit 1; }
    echo "rep $rep $T: $(python -c "import json;d=json.load(open('$OUT/bench_${T}_$rep.json'));print(d['ms_per_step'], d['value'])")"
  done
done
