set -u
bash tools/parity_variants.sh gpurun_out/r04i lbt_amd/liblbt_dfxp.so || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "head or deeper or evaluate or partial" tests/test_igemm_big.py tests/test_resnet50.py > gpurun_out/r04i/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04i/tests.log; [ $rc -le 1 ] || exit $rc
bash tools/ab_env.sh gpurun_out/r04i 3 "LBT_HEAD_CHAIN=1" "LBT_HEAD_CHAIN=0" || exit 1
bash tools/ab_bench.sh gpurun_out/r04i_r50 2 lbt_amd/liblbt_dfxp.so lbt_amd/build_var/plain/liblbt_dfxp.so -- --workload resnet50 --steps 20 --warmup 5
