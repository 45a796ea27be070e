cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread --deselect tests/test_bench_shared_gpu.py::test_bench_multi_rank_on_one_gpu > gpurun_out/pytest_gpu_rest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_rest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_bench_shared_gpu.py -x -v --timeout 500 --timeout-method thread > gpurun_out/pytest_gpu_bsg.log 2>&1; rc=$?
echo "bench_shared rc=$rc"; tail -3 gpurun_out/pytest_gpu_bsg.log; exit $rc
