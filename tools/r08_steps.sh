set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r08
timeout -k 10 500 python -u -m pytest tests/test_dp_gpu.py tests/test_dp_resnet50_gpu.py tests/test_edge_cases.py -m gpu -v --timeout 240 \
  --timeout-method thread > gpurun_out/r08/dp_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r08/dp_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r08/smoke.log 2>&1; rc=$?
tail -1 gpurun_out/r08/smoke.log; [ $rc = 0 ] || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r08/bench.json 2> gpurun_out/r08/bench.err; rc=$?
cat gpurun_out/r08/bench.json | cut -c1-400; [ $rc = 0 ] || exit 1
echo done
