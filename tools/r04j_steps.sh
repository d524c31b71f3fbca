set -u
mkdir -p gpurun_out/r04j
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04j/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04j/gpu_tests.log; [ $rc -le 1 ] || exit $rc
bash tools/ab_bench.sh gpurun_out/r04j_r50 2 lbt_amd/liblbt_dfxp.so lbt_amd/build_var/plain/liblbt_dfxp.so -- --workload resnet50 --steps 20 --warmup 5
