#!/bin/bash
# A/B of the 256-row LDS-DMA igemm (igemm_big_kernel) on the GPU box: parity first (the igemm /
# ResNet-50 GPU tests with the big kernel forced onto every eligible GEMM, LBT_IGEMM_BIG_MIN=1),
# then tools/igemm_probe.py with the big kernel on and off.  -> gpurun_out/igab/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/igab; mkdir -p $OUT
LBT_IGEMM_BIG_MIN=1 timeout -k 10 400 python -u -m pytest tests/test_resnet50.py -x -q --timeout 200 --timeout-method thread > $OUT/tests_forced.log 2>&1
rc=$?; tail -2 $OUT/tests_forced.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/igemm_probe.py > $OUT/probe_big.txt 2>&1 || exit 1
LBT_IGEMM_BIG=0 timeout -k 10 200 python tools/igemm_probe.py > $OUT/probe_old.txt 2>&1 || exit 1
paste <(awk '{print $1, $2}' $OUT/probe_old.txt) <(awk '{print $2, $NF-0, $0}' $OUT/probe_big.txt | cut -c1-20) | grep -v amdgpu
