set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04z
timeout -k 10 300 python -u -m pytest tests/test_resnet50.py -m gpu -v --timeout 240 -k "stem" \
  --timeout-method thread > gpurun_out/r04z/first.log 2>&1; rc=$?
tail -3 gpurun_out/r04z/first.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python tools/stem_probe.py > gpurun_out/r04z/stem_probe.txt 2>&1; rc=$?
cat gpurun_out/r04z/stem_probe.txt; [ $rc = 0 ] || exit 1
bash tools/ab_env.sh gpurun_out/r04z_r50 2 "LBT_STEM_CG=32" "LBT_STEM_CG=64" -- --workload resnet50 --steps 20 --warmup 5 || exit 1
echo done
