#!/bin/bash
# The B=128 fused-plan oracle test against several library builds (scratch A/B builds):
#   tools/parity_variants.sh OUT LIB1 [LIB2 ...]
# A test failure (exit 1) goes on to the next build; anything else (a crash, a time limit) stops.
set -u
OUT=$1; shift
mkdir -p "$OUT"
for L in "$@"; do
  T=$(basename "$(dirname "$L")"); [ "$T" = lbt_amd ] && T=main
  LBT_LIBRARY=$(realpath "$L") timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "tests/test_gpu_parity.py::test_fused_bench_workload_bitexact_vs_oracle" > "$OUT/parity_$T.log" 2>&1
  rc=$?
  echo "$T: rc=$rc $(tail -1 "$OUT/parity_$T.log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
