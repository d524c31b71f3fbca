set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04q
timeout -k 10 300 python -u -m pytest tests/test_igemm_big.py -m gpu -v --timeout 240 -k "bna or bn3" \
  --timeout-method thread > gpurun_out/r04q/first.log 2>&1; rc=$?
tail -3 gpurun_out/r04q/first.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python tools/bna_probe.py > gpurun_out/r04q/bna_probe.txt 2>&1; rc=$?
cat gpurun_out/r04q/bna_probe.txt; [ $rc = 0 ] || exit 1
PROBE_ONLY=l1_c2_fwd,l2_c2_fwd,l3_c2_fwd,l4_c2_fwd,l1_c2_fwdq,l2_c2_fwdq,l3_c2_fwdq PROBE_QNOISE=table timeout -k 10 240 python tools/igemm_probe.py > gpurun_out/r04q/probe.txt 2>&1; cat gpurun_out/r04q/probe.txt
echo done
