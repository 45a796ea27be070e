#!/bin/bash
# Network-kernel probe: phase stamps (c3, c4; ablations), then PMC passes of
# tools/kernel_bench.py c3 with instruction-cache and issue counters.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/np
timeout -k 10 120 python3 tools/net_stamps.py c3 0,1,64 > gpurun_out/np/stamps_c3.txt 2>&1 || exit 5
timeout -k 10 120 python3 tools/net_stamps.py c4 0 > gpurun_out/np/stamps_c4.txt 2>&1 || exit 5
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/np/avail.txt 2>&1
grep -o -E "SQC_[A-Z_]*|SQ_IFETCH[A-Z_]*|SQ_WAIT_INST[A-Z_]*|SQ_INST_LEVEL[A-Z_]*|SQ_INSTS_[A-Z_]*" gpurun_out/np/avail.txt | sort -u > gpurun_out/np/names.txt
CMD="python3 tools/kernel_bench.py c3 50"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d gpurun_out/np/p1 -o p1 -- $CMD > gpurun_out/np/p1.log 2>&1; echo p1 rc=$?
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA --output-format csv -d gpurun_out/np/p2 -o p2 -- $CMD > gpurun_out/np/p2.log 2>&1; echo p2 rc=$?
exit 0
