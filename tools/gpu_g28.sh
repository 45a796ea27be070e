#!/bin/bash
# The segmented sample on row-pair units (eight-wave workgroups, 256 runs):
# its tests, kernel timing at C4 one GPU and a W = 8 rank, rank timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
mkdir -p gpurun_out/g28
timeout -k 10 600 python -u -m pytest tests/test_hip_kstream.py tests/test_hip_lds_poison.py tests/test_hip_sharded_run.py tests/test_hip_fullsize.py tests/test_hip_parity.py -x -q --timeout 180 --timeout-method thread > gpurun_out/g28/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/g28/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  timeout -k 10 200 python3 tools/kernel_bench.py c4 20 35=$v > gpurun_out/g28/kb_c4_$v.txt 2>&1 || exit 5
  tail -1 gpurun_out/g28/kb_c4_$v.txt
done
timeout -k 10 300 python3 tools/rank_timing.py --cfg c4 --world 8 --schedule run > gpurun_out/g28/rank_w8.jsonl 2>&1 || { tail -5 gpurun_out/g28/rank_w8.jsonl; exit 6; }
tail -1 gpurun_out/g28/rank_w8.jsonl
exit 0
