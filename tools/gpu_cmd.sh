#!/bin/bash
# scratch GPU session script (edited per call)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/t4.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 8 gpurun_out/t4.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python3 tools/net_stamps.py c3 > gpurun_out/ns_c3.log 2>&1; echo "stamps rc=$?"; grep -v realtime gpurun_out/ns_c3.log | head -16
timeout -k 10 120 python3 tools/net_stamps.py c3 0 8 0 > gpurun_out/ns_c3w8.log 2>&1; echo "stamps8 rc=$?"; grep -v realtime gpurun_out/ns_c3w8.log | head -16
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-trainers --no-lenet > gpurun_out/b2.log 2>&1; echo bench rc=$?; tail -c 900 gpurun_out/b2.log
timeout -k 10 200 python -u tools/rank_timing.py --cfg c4 --world 8 --ranks 0,4 > gpurun_out/rt_c4b.log 2>&1; echo "rt rc=$?"; tail -n 3 gpurun_out/rt_c4b.log
timeout -k 10 200 python -u tools/rank_timing.py --cfg weak --world 8 --ranks 0,4 > gpurun_out/rt_wb.log 2>&1; echo "rt rc=$?"; tail -n 3 gpurun_out/rt_wb.log
CMD="python3 tools/rank_timing.py --cfg c4 --world 8 --ranks 0 --iters 10 --warmup 2" \
PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY|SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
  bash tools/pmc_session.sh; echo "pmc rc=$?"
python3 tools/pmc_report.py gpurun_out/pmc > gpurun_out/pmc_rank.txt 2>&1; grep -A16 "== mvn_kstream\|== mvn_fwd_kernel\|== net_kernel" gpurun_out/pmc_rank.txt | head -60
