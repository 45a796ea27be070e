#!/bin/bash
# The HVP sample pair on one paired bf16-piece launch (PSVI_DBG_FWD_PAIR_BF 2):
# the HVP tests, C3 psvi_hvp timing per form, kernel stats of the paired form.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
mkdir -p gpurun_out/g26
timeout -k 10 300 python -u -m pytest tests/test_hip_hvp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g26/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/g26/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 2 3; do
    timeout -k 10 120 python3 tools/hvp_probe.py --n 200 --dbg 31=$v 2>&1 | grep "mixed=True" || exit 3
  done
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g26/tr2 -o t -- python3 tools/hvp_probe.py --n 100 --dbg 31=2 > gpurun_out/g26/tr2.log 2>&1 || exit 4
f=$(ls gpurun_out/g26/tr2/*/t_kernel_stats.csv 2>/dev/null || find gpurun_out/g26/tr2 -name "*kernel_stats.csv" | head -1)
cut -d, -f1-5 $(find gpurun_out/g26/tr2 -name "*kernel_stats.csv" | head -1) | head -12
exit 0
