# ResNet-50 layer path: wgrad slab reduces + BN parameter gradients batched (LBT_BATCH_WREDUCE / _PGRADS)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s10; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resnet50.py tests/test_dp_resnet50_gpu.py -m gpu > $O/parity.log 2>&1 || { echo parity failed; tail -5 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for rep in 1 2; do
  for E in 0 1; do
    LBT_BATCH_WREDUCE=$E LBT_BATCH_PGRADS=$E timeout -k 10 200 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $O/r50_${E}_$rep.json 2>/dev/null || exit 1
    echo "R50 rep $rep batched=$E $(python -c "import json;print(json.load(open('$O/r50_${E}_$rep.json'))['ms_per_step'])")"
  done
done
