#!/bin/bash
# Round-end evidence in one gpurun call: GPU tests, smoke, bench (JSON line),
# rocprofv3 kernel trace of the bench, PMC HBM-traffic passes of the bench.
# Stops at the first crash / abort / timeout (rc not in {0,1}).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
R=${ROUND:-r01}
STEPS=${STEPS:-tests,smoke,bench,prof,lprof,pmc,lpmc}
if [[ ,$STEPS, == *,tests,* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
fi
if [[ ,$STEPS, == *,smoke,* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; ok $rc || exit $rc
fi
if [[ ,$STEPS, == *,bench,* ]]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench_${R}.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 gpurun_out/bench_${R}.log; ok $rc || exit $rc
fi
BCMD="python3 bench.py --no-cpu-baseline --no-trainers --no-lenet --no-c4 --no-c2 --steps 200 --warmup 20"
if [[ ,$STEPS, == *,prof,* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${R} -o bench -- $BCMD > gpurun_out/prof_${R}.log 2>&1; rc=$?
  echo "prof rc=$rc"; ok $rc || exit $rc
fi
if [[ ,$STEPS, == *,lprof,* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof_${R} -o lenet -- python3 tools/lenet_probe.py --T 5 --reps 1 > gpurun_out/lprof_${R}.log 2>&1; rc=$?
  echo "lenet prof rc=$rc"; ok $rc || exit $rc
fi
if [[ ,$STEPS, == *,pmc,* ]]; then
  CMD="python3 bench.py --no-cpu-baseline --no-trainers --no-lenet --no-c4 --no-c2 --steps 50 --warmup 5" \
  PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS|SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY|SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
    bash tools/pmc_session.sh; rc=$?
  echo "pmc rc=$rc"; ok $rc || exit $rc
  python3 tools/pmc_report.py gpurun_out/pmc --json gpurun_out/pmc_traffic_${R}.json > gpurun_out/pmc_report_${R}.txt 2>&1
  tail -30 gpurun_out/pmc_report_${R}.txt
fi
if [[ ,$STEPS, == *,lpmc,* ]]; then
  mkdir -p gpurun_out/lpmc_${R}
  timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/lpmc_${R} -o lenet -- python3 tools/lenet_probe.py --T 2 --reps 1 > gpurun_out/lpmc_${R}.log 2>&1; rc=$?
  echo "lenet pmc rc=$rc"; ok $rc || exit $rc
fi
exit 0
