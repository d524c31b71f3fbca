#!/bin/bash
# usage: tools/gpu_retry.sh OUTFILE TIMEOUT 'command'  -- re-issues only when no box was obtained (nothing ran)
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 ${GPU_RETRIES:-30}); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  if grep -q "status=transient" "$OUT" && grep -q "run 0.0s\|run Nones" "$OUT"; then
    sleep 150; continue
  fi
  break
done
