# 2-row tiles for the 16-channel stage too (B = 16): parity, then A/B vs LBT_TILE_ROWS1=4
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s8; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_int4.py tests/test_dp_gpu.py -m gpu -k "fused or golden or timed or int4 or w4 or world" > $O/parity.log 2>&1 || { echo parity failed; tail -5 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for rep in 1 2 3; do
  for E in 4 0; do
    LBT_TILE_ROWS1=$E timeout -k 10 120 python bench.py --batch 16 --steps 400 --warmup 40 --no-cpu-baseline --no-roofline > $O/b16_${E}_$rep.json 2>/dev/null || exit 1
    echo "B16 rep $rep rows1=$E $(python -c "import json;print(json.load(open('$O/b16_${E}_$rep.json'))['ms_per_step'])")"
  done
done
