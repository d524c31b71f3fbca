set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04y
timeout -k 10 300 python -u -m pytest tests/test_resnet50.py -m gpu -v --timeout 240 -k "stem or bottleneck or resnet50" \
  --timeout-method thread > gpurun_out/r04y/first.log 2>&1; rc=$?
tail -3 gpurun_out/r04y/first.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python tools/stem_probe.py > gpurun_out/r04y/stem_probe.txt 2>&1; rc=$?
cat gpurun_out/r04y/stem_probe.txt; [ $rc = 0 ] || exit 1
bash tools/ab_env.sh gpurun_out/r04y_r50 2 "LBT_STEM_ROWS=1" "LBT_STEM_ROWS=0" -- --workload resnet50 --steps 20 --warmup 5 || exit 1
echo done
