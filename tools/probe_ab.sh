#!/bin/bash
# igemm per-shape probe (tools/igemm_probe.py) against several library builds: tools/probe_ab.sh OUT SHAPES LIB...
set -uo pipefail
OUT=$1; SHAPES=$2; shift 2
mkdir -p "$OUT"
for L in "$@"; do
  T=$(basename "$(dirname "$L")"); [ "$T" = lbt_amd ] && T=main
  LBT_LIBRARY=$(realpath "$L") PROBE_ONLY=$SHAPES PROBE_QNOISE=table timeout -k 10 240 python tools/igemm_probe.py > "$OUT/probe_$T.txt" 2>&1 || { echo "probe $T failed"; tail -3 "$OUT/probe_$T.txt"; exit 1; }
  echo "== $T"; cat "$OUT/probe_$T.txt"
done
