# ResNet-50 layer path: BN parameter gradients batched into one launch (LBT_BATCH_PGRADS): parity, then A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s9; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resnet50.py -m gpu -k "deferred or full_size or side_stream or bitexact_vs_oracle and 16" > $O/parity.log 2>&1 || { echo parity failed; tail -5 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for rep in 1 2; do
  for E in 0 1; do
    LBT_BATCH_PGRADS=$E timeout -k 10 200 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $O/r50_${E}_$rep.json 2>/dev/null || exit 1
    echo "R50 rep $rep batch_pgrads=$E $(python -c "import json;print(json.load(open('$O/r50_${E}_$rep.json'))['ms_per_step'])")"
  done
done
