#!/bin/bash
# One gpurun check: selected GPU tests (TESTS, default all), then optionally
# a quick bench line and its rocprofv3 kernel stats (BENCH=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-trainers --no-lenet --no-c4 --no-c2 --steps 500 --warmup 30 > gpurun_out/bench_q.log 2>&1; rc=$?; tail -1 gpurun_out/bench_q.log | cut -c1-300; [ $rc -le 1 ] || exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q -o bench -- python3 bench.py --no-cpu-baseline --no-trainers --no-lenet --no-c4 --no-c2 --steps 200 --warmup 20 > gpurun_out/prof_q.log 2>&1; echo prof rc=$?
fi
exit 0
