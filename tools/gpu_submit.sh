#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool had no box / slot for it (the call ended
# "transient" with nothing charged: no part of the command ran). A call that ran -- whatever its
# result -- is never repeated.
#   tools/gpu_submit.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 ${GPU_SUBMIT_TRIES:-20}); do
  timeout $((TO + 1200)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  if grep -q "status=transient" "$OUT" && grep -q "charged=0.0s\|charged=Nones" "$OUT"; then
    sleep ${GPU_SUBMIT_WAIT:-120}
    continue
  fi
  break
done
