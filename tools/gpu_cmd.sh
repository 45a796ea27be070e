#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 30 ./tools/probes/buf_oob > gpurun_out/oob.log 2>&1; cat gpurun_out/oob.log
timeout -k 10 200 python -u tools/sharded_debug.py 2 256 100 3 > gpurun_out/sd.log 2>&1; echo "sd rc=$?"; tail -n 30 gpurun_out/sd.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t5.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 15 gpurun_out/t5.log
