set -u
CHECK_DP=0 bash tools/gpu_check.sh r04n || exit 1
bash tools/probe_ab.sh gpurun_out/r04n_probe l1_c2_fwdq,l2_c2_fwdq,l3_c2_fwdq,l1_c3_fwdq,l3_c3_fwdq,l1_c2_fwd,l3_c2_fwd,l1_c2_dgrad16,l3_c2_dgrad16,l1_c3_dgrad16,l1_c1_dgrad16 lbt_amd/liblbt_dfxp.so lbt_amd/build_var/prevq/liblbt_dfxp.so || exit 1
bash tools/ab_bench.sh gpurun_out/r04n_r50 1 lbt_amd/liblbt_dfxp.so lbt_amd/build_var/prevq/liblbt_dfxp.so -- --workload resnet50 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04n_fetchcal -o run -- tools/fetch_cal > gpurun_out/r04n_fetchcal.log 2>&1
