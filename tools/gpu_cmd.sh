#!/bin/bash
# scratch GPU session script (edited per call)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 15 gpurun_out/t2.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rtprof -o rt -- python3 tools/rank_timing.py --cfg c4 --world 8 --ranks 0,4 --iters 30 > gpurun_out/rt_prof.log 2>&1; echo "rtprof rc=$?"
