#!/bin/bash
# One GPU-box pass over the current build (run from the repo root via gpurun):
#   tools/gpu_check.sh <tag>
# -> gpurun_out/check_<tag>/: the -m gpu suite log, smoke, the default bench line, and a 2-rank
#    rehearsal of the launcher (gloo, both ranks on the one GPU) for weak and strong scaling.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -euo pipefail
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/check_$TAG
rm -rf "$OUT" && mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$OUT/gpu_tests.log" 2>&1
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
if [ "${CHECK_DP:-1}" = 1 ]; then
  LBT_DIST_BACKEND=gloo LBT_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 3 \
    --no-cpu-baseline --no-roofline > "$OUT/dp2_weak.json" 2> "$OUT/dp2_weak.err"
  cat "$OUT/dp2_weak.json"
  LBT_DIST_BACKEND=gloo LBT_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --global-batch 128 --steps 20 \
    --warmup 3 --no-cpu-baseline --no-roofline > "$OUT/dp2_strong.json" 2> "$OUT/dp2_strong.err"
  cat "$OUT/dp2_strong.json"
fi
echo "all done"
