#!/bin/bash
# Round-6 evidence in one gpurun call: round_session.sh's steps (GPU suite,
# smoke, bench, rocprof kernel stats of the bench and of LeNet, PMC passes of
# the bench, LeNet PMC), then the network kernel's stamps at C3, the W = 8
# rank timing and the overlap timing.  Stops at the first crash / timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
ROUND=r06 STEPS=${STEPS:-tests,smoke,bench,prof,lprof,pmc,lpmc} bash tools/round_session.sh || exit $?
if [[ ,${EXTRA:-stamps,rank,overlap}, == *,stamps,* ]]; then
  timeout -k 10 120 python3 tools/net_stamps.py c3 > gpurun_out/r06/net_stamps_c3.txt 2>&1 || { tail -5 gpurun_out/r06/net_stamps_c3.txt; exit 5; }
  timeout -k 10 120 python3 tools/net_stamps.py c4 > gpurun_out/r06/net_stamps_c4.txt 2>&1 || { tail -5 gpurun_out/r06/net_stamps_c4.txt; exit 5; }
fi
if [[ ,${EXTRA:-stamps,rank,overlap}, == *,rank,* ]]; then
  timeout -k 10 300 python3 tools/rank_timing.py --cfg c4 --world 8 --schedule run > gpurun_out/r06/rank_timing_w8_run.jsonl 2>&1 || { tail -5 gpurun_out/r06/rank_timing_w8_run.jsonl; exit 6; }
  tail -1 gpurun_out/r06/rank_timing_w8_run.jsonl
fi
if [[ ,${EXTRA:-stamps,rank,overlap}, == *,overlap,* ]]; then
  timeout -k 10 300 python3 tools/overlap_timing.py --world 8 --rank 0 --delays 0,10,20,40 --T 30 > gpurun_out/r06/overlap_w8.jsonl 2>&1 || { tail -5 gpurun_out/r06/overlap_w8.jsonl; exit 7; }
fi
exit 0
