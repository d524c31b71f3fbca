set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
bash tools/ab_env.sh gpurun_out/r09_fq 3 "LBT_FUSE_CONV_QUANT=2" "LBT_FUSE_CONV_QUANT=1" -- --workload resnet50 --steps 30 --warmup 5 || exit 1
echo done
