#!/bin/bash
# scratch GPU session script (edited per call)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/t4.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 8 gpurun_out/t4.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python3 tools/net_stamps.py c3 > gpurun_out/ns_c3.log 2>&1; echo "stamps rc=$?"; head -30 gpurun_out/ns_c3.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-trainers --no-lenet > gpurun_out/b2.log 2>&1; echo bench rc=$?; tail -c 900 gpurun_out/b2.log
