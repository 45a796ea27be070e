#!/bin/bash
# W = 8 rank timing, the segmented sample's row-pair form against the 64-row
# one (PSVI_DBG_FWD_ROWS_OFF 35), alternating on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
mkdir -p gpurun_out/g29
for v in 1 0 1 0; do
  timeout -k 10 300 python3 tools/rank_timing.py --cfg c4 --world 8 --schedule run --dbg 35=$v > gpurun_out/g29/rank_w8_$v.jsonl 2>&1 || { tail -5 gpurun_out/g29/rank_w8_$v.jsonl; exit 6; }
  echo "35=$v $(tail -1 gpurun_out/g29/rank_w8_$v.jsonl)"
  grep '"rank": 0' gpurun_out/g29/rank_w8_$v.jsonl
done
exit 0
