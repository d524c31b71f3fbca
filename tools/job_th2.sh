# 2-row tiles of the 32-/64-channel fused conv kernels: parity (fused plan vs oracle, golden fixtures,
# int4) then an interleaved A/B against LBT_TILE_ROWS23=4 (the former 4-row tiles) at B=128 and B=16
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s6; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_int4.py -m gpu -k "fused or golden or timed or int4 or w4" > $O/parity_th2.log 2>&1 || { echo parity failed; tail -5 $O/parity_th2.log; exit 1; }
tail -2 $O/parity_th2.log
for rep in 1 2 3; do
  for E in 4 0; do
    LBT_TILE_ROWS23=$E timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-roofline > $O/b128_${E}_$rep.json 2>/dev/null || exit 1
    echo "B128 rep $rep rows23=$E $(python -c "import json;print(json.load(open('$O/b128_${E}_$rep.json'))['ms_per_step'])")"
  done
done
for rep in 1 2; do
  for E in 4 0; do
    LBT_TILE_ROWS23=$E timeout -k 10 120 python bench.py --batch 16 --steps 400 --warmup 40 --no-cpu-baseline --no-roofline > $O/b16_${E}_$rep.json 2>/dev/null || exit 1
    echo "B16 rep $rep rows23=$E $(python -c "import json;print(json.load(open('$O/b16_${E}_$rep.json'))['ms_per_step'])")"
  done
done
