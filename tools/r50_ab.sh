#!/bin/bash
# ResNet-50 (configs[3]) bench A/B over env variants -> gpurun_out/r50ab/<tag>.json
#   bash tools/r50_ab.sh "base:" "fq:LBT_FUSE_CONV_QUANT=1" ...   (default: big igemm on / off)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r50ab; mkdir -p $OUT
[ $# -gt 0 ] || set -- "big:" "old:LBT_IGEMM_BIG=0"
for v in "$@"; do
  tag=${v%%:*}; envs=${v#*:}
  env ${envs//,/ } timeout -k 10 400 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err || exit 1
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag',d['ms_per_step'],d['config'].get('final_loss'))"
done
