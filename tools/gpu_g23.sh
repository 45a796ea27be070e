cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g23 && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; grep -E "^FAILED" gpurun_out/pytest_gpu.log | head; exit $rc
