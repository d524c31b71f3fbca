set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06
CHECK_DP=0 bash tools/gpu_check.sh r06 || exit 1
LBT_HEAD=909d777 bash tools/profile_round.sh r06 || exit 1
LBT_HEAD=909d777 bash tools/profile_round.sh r06_r50 --workload resnet50 --steps 20 --warmup 5 || exit 1
timeout -k 10 200 python tools/stem_probe.py > gpurun_out/r06/stem_probe.txt 2>&1; cat gpurun_out/r06/stem_probe.txt
LBT_FUSE_CONV_QUANT=2 timeout -k 10 300 python -u -m pytest tests/test_resnet50.py tests/test_igemm_big.py -m gpu -q --timeout 240 \
  --timeout-method thread -k "bottleneck or resnet50" > gpurun_out/r06/fuseq2_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06/fuseq2_tests.log; [ $rc = 0 ] || exit 1
bash tools/ab_env.sh gpurun_out/r06_fq 2 "LBT_FUSE_CONV_QUANT=2" "LBT_FUSE_CONV_QUANT=1" -- --workload resnet50 --steps 20 --warmup 5 || exit 1
echo done
