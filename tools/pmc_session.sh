#!/bin/bash
# Kernel trace + PMC counter passes (one rocprofv3 run per counter group; no
# sys/runtime tracing mixed with --pmc).  Writes under gpurun_out/pmc/.
#   CMD=...          profiled command (default: tools/kernel_bench.py $CFG)
#   PMC_GROUPS=...   counter groups separated by '|', counters within a group by spaces
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf gpurun_out/pmc
mkdir -p gpurun_out/pmc
CFG=${CFG:-c3}
CMD=${CMD:-"python3 tools/kernel_bench.py $CFG ${ITERS:-50}"}
GROUPS_STR=${PMC_GROUPS:-"FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS|SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY|TCC_HIT_sum TCC_MISS_sum|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/trace -o trace -- $CMD > gpurun_out/pmc/trace.log 2>&1 || exit $?
IFS='|' read -r -a GRPS <<< "$GROUPS_STR"
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o p$i -- $CMD > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pmc group $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || tail -3 gpurun_out/pmc/p$i.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
exit 0
