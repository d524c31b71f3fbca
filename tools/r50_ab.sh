#!/bin/bash
# ResNet-50 (configs[3]) bench with the 256-row LDS-DMA igemm on (default) and off -> gpurun_out/r50ab/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r50ab; mkdir -p $OUT
timeout -k 10 400 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/big.json 2> $OUT/big.err || exit 1
python -c "import json;d=json.load(open('$OUT/big.json'));print('big',d['ms_per_step'],d['config'].get('final_loss'))"
LBT_IGEMM_BIG=0 timeout -k 10 400 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/old.json 2> $OUT/old.err || exit 1
python -c "import json;d=json.load(open('$OUT/old.json'));print('old',d['ms_per_step'],d['config'].get('final_loss'))"
