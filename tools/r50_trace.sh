#!/bin/bash
# ResNet-50 (configs[3]) kernel trace of a short bench run -> gpurun_out/r50t/<tag>/ (+ per-shape summary)
#   bash tools/r50_trace.sh <tag> [ENV=VAL ...]
set -euo pipefail
TAG=${1:?tag}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r50t/$TAG; rm -rf $OUT; mkdir -p $OUT
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python bench.py --workload resnet50 --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > $OUT/log 2>&1
python tools/r50_shapes.py $OUT/run_kernel_trace.csv > $OUT/shapes.txt && head -60 $OUT/shapes.txt
