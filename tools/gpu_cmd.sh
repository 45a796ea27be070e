#!/bin/bash
# scratch GPU session script (edited per call)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_hip_kstream.py tests/test_hip_parity.py tests/test_hip_variants.py tests/test_hip_stream.py -q --timeout 240 --timeout-method thread > gpurun_out/t3.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 8 gpurun_out/t3.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python3 tools/net_stamps.py c3 > gpurun_out/ns_c3.log 2>&1; echo "stamps rc=$?"; cat gpurun_out/ns_c3.log | head -40
