set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r10w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/r10w/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r10w/gpu_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r10w/smoke.log 2>&1; rc=$?
tail -1 gpurun_out/r10w/smoke.log; [ $rc = 0 ] || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r10w/bench.json 2> gpurun_out/r10w/bench.err; rc=$?
cut -c1-600 gpurun_out/r10w/bench.json; [ $rc = 0 ] || exit 1
timeout -k 10 400 python bench.py --workload resnet50 --steps 20 --warmup 5 > gpurun_out/r10w/bench_r50.json 2> gpurun_out/r10w/bench_r50.err; rc=$?
cut -c1-400 gpurun_out/r10w/bench_r50.json; [ $rc = 0 ] || exit 1
echo done
