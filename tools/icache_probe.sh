cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ic && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/ic/avail.txt 2>&1; echo list rc=$?
grep -o -E "SQC_ICACHE[A-Z_]*|SQ_IFETCH[A-Z_]*|SQC_TC_INST[A-Z_]*|SQ_INST_LEVEL[A-Z_]*|SQ_WAIT_INST[A-Z_]*" gpurun_out/ic/avail.txt | sort -u > gpurun_out/ic/names.txt; cat gpurun_out/ic/names.txt
CMD="python3 bench.py --no-cpu-baseline --no-trainers --no-lenet --no-c4 --no-c2 --steps 50 --warmup 5"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d gpurun_out/ic/p1 -o p1 -- $CMD > gpurun_out/ic/p1.log 2>&1; echo p1 rc=$?
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/ic/p2 -o p2 -- $CMD > gpurun_out/ic/p2.log 2>&1; echo p2 rc=$?
exit 0
