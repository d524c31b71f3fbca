# 2-row tiles where the 32-/64-channel launches have fewer tiles than CUs: parity, then A/B per batch
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s7; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_int4.py tests/test_dp_gpu.py -m gpu -k "fused or golden or timed or int4 or w4 or world" > $O/parity_th2b.log 2>&1 || { echo parity failed; tail -5 $O/parity_th2b.log; exit 1; }
tail -2 $O/parity_th2b.log
for B in 16 32 64 128; do
  for rep in 1 2; do
    for E in 4 0; do
      LBT_TILE_ROWS23=$E timeout -k 10 120 python bench.py --batch $B --steps 400 --warmup 40 --no-cpu-baseline --no-roofline > $O/b${B}_${E}_$rep.json 2>/dev/null || exit 1
      echo "B$B rep $rep rows23=$E $(python -c "import json;print(json.load(open('$O/b${B}_${E}_$rep.json'))['ms_per_step'])")"
    done
  done
done
