set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06
CHECK_DP=0 bash tools/gpu_check.sh r06 || exit 1
LBT_HEAD=909d777 bash tools/profile_round.sh r06 || exit 1
LBT_HEAD=909d777 bash tools/profile_round.sh r06_r50 --workload resnet50 --steps 20 --warmup 5 || exit 1
timeout -k 10 200 python tools/stem_probe.py > gpurun_out/r06/stem_probe.txt 2>&1; cat gpurun_out/r06/stem_probe.txt
echo done
