#!/bin/bash
# The K-split kernel keeping a band's G rows across same-band tiles: its tests,
# C3 psvi_hvp timing, kernel stats, C4 one-GPU loop timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
mkdir -p gpurun_out/g27
timeout -k 10 600 python -u -m pytest tests/test_hip_hvp.py tests/test_hip_kstream.py tests/test_hip_sharded_run.py tests/test_hip_hypergrad.py -x -q --timeout 180 --timeout-method thread > gpurun_out/g27/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/g27/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python3 tools/hvp_probe.py --n 200 2>&1 | grep "mixed=True" || exit 3
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g27/tr -o t -- python3 tools/hvp_probe.py --n 100 > gpurun_out/g27/tr.log 2>&1 || exit 4
timeout -k 10 200 python3 tools/kernel_bench.py c4 20 > gpurun_out/g27/kb_c4.txt 2>&1 || exit 5
tail -12 gpurun_out/g27/kb_c4.txt
exit 0
