set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s4; mkdir -p $O
LBT_DEFER_UNDERFILLED=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "fused_bench_workload_bitexact" > $O/parity_defer.log 2>&1 || { echo parity failed; exit 1; }
tail -2 $O/parity_defer.log
for rep in 1 2 3; do
  for E in 0 1; do
    LBT_DEFER_UNDERFILLED=$E timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-roofline > $O/b128_${E}_$rep.json 2>/dev/null || exit 1
    echo "B128 rep $rep defer=$E $(python -c "import json;print(json.load(open('$O/b128_${E}_$rep.json'))['ms_per_step'])")"
  done
done
for rep in 1 2; do
  for E in 0 1; do
    LBT_DEFER_UNDERFILLED=$E timeout -k 10 120 python bench.py --batch 16 --steps 400 --warmup 40 --no-cpu-baseline --no-roofline > $O/b16_${E}_$rep.json 2>/dev/null || exit 1
    echo "B16 rep $rep defer=$E $(python -c "import json;print(json.load(open('$O/b16_${E}_$rep.json'))['ms_per_step'])")"
  done
done
