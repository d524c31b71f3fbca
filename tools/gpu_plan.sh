#!/bin/bash
# One parameterised GPU-box job (run from the repo root via gpurun). Replaces the per-round
# tools/r0*_steps.sh job lists.
#
#   tools/gpu_plan.sh <tag> <step> [<step> ...]
#
# Steps (each under its own time limit; the chain stops at the first failure, so nothing more runs
# on the GPU after a fault, an abort or a time-out):
#   tests            the whole -m gpu suite
#   tests:<path>[:<k>]  a subset: tests:tests/test_gpu_parity.py  or  tests:tests:fused or golden
#   smoke            __graft_entry__.smoke()
#   bench[:args]     bench.py (default arguments, or the ':'-separated extra ones, e.g. bench:--batch:16)
#   r50              bench.py --workload resnet50 --steps 20 --warmup 5
#   trace:<B>        rocprofv3 kernel trace of the graph-replayed fused step at per-GPU batch B, summarised
#                    per launch position (tools/step_positions.py)
#   strong           tools/strong_probe.py (per-GPU batch 16/32/64/128 + world-1 RCCL exchange)
#   py:<script>[:args]  python <script> args
# Any step may carry environment settings for its own run: VAR=val+VAR2=val@<step>
# Output: gpurun_out/<tag>/
set -u
TAG=${1:?tag}
shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
n=0
run_step() {
  case "$name" in
    tests)
      # tests[:<path>[:<-k expression>]]
      sel="tests"; kx=""
      if [ -n "$rest" ]; then sel=${rest%%:*}; [ "$rest" != "$sel" ] && kx=${rest#*:}; fi
      if [ -n "$kx" ]; then
        timeout -k 10 900 python -u -m pytest $sel -m gpu -x -q --timeout 240 --timeout-method thread -k "$kx" \
          > "$log.log" 2>&1; rc=$?
      else
        timeout -k 10 900 python -u -m pytest $sel -m gpu -x -q --timeout 240 --timeout-method thread \
          > "$log.log" 2>&1; rc=$?
      fi
      tail -3 "$log.log" ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$log.log" 2>&1; rc=$?
      tail -1 "$log.log" ;;
    bench)
      timeout -k 10 400 python bench.py $args > "$log.json" 2> "$log.err"; rc=$?
      cut -c1-700 "$log.json" ;;
    r50)
      timeout -k 10 400 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu-baseline $args \
        > "$log.json" 2> "$log.err"; rc=$?
      cut -c1-400 "$log.json" ;;
    trace)
      B=${args:-128}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$log" -o run -- \
        python bench.py --batch "$B" --steps 60 --warmup 10 --no-cpu-baseline --no-roofline > "$log.log" 2>&1; rc=$?
      if [ $rc = 0 ]; then
        csv=$(find "$log" -name '*kernel_trace.csv' | head -1)
        python tools/step_positions.py "$csv" 10 > "$log.positions.txt" 2>&1 || true
        tail -1 "$log.positions.txt"
      fi ;;
    strong)
      timeout -k 10 600 python tools/strong_probe.py $args --out "$log.json" > "$log.log" 2>&1; rc=$?
      tail -2 "$log.log" ;;
    py)
      timeout -k 10 600 python $args > "$log.log" 2>&1; rc=$?
      tail -5 "$log.log" ;;
    *)
      echo "unknown step $step"; rc=2 ;;
  esac
  return $rc
}
for step in "$@"; do
  n=$((n + 1))
  envs=()
  if [[ "$step" == *@* ]]; then
    # VAR=val+VAR2=val: a '+' piece without '=' belongs to the previous value (e.g. PROBE_ONLY=a+b,c+d)
    IFS='+' read -ra parts <<< "${step%%@*}"
    for pc in "${parts[@]}"; do
      if [[ "$pc" == *=* || ${#envs[@]} -eq 0 ]]; then envs+=("$pc"); else envs[-1]="${envs[-1]}+$pc"; fi
    done
    step=${step#*@}
  fi
  name=${step%%:*}
  rest=""
  [ "$step" != "$name" ] && rest=${step#*:}
  args=${rest//:/ }
  log="$OUT/$(printf %02d $n)_${name}"
  [ ${#envs[@]} -gt 0 ] && printf '%s\n' "${envs[@]}" > "$log.env"
  ( for ev in "${envs[@]}"; do export "$ev"; done; run_step ); rc=$?
  if [ $rc != 0 ]; then
    echo "step $step failed rc=$rc"; exit 1
  fi
done
echo "all done"
