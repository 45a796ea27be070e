#!/bin/bash
# One gpurun session: GPU tests -> bench -> rocprofv3 kernel trace.
# Stops issuing GPU work after any crash / abort / timeout (rc not in {0,1}).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
STEPS=${STEPS:-tests,bench,prof}
rc=0
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -m gpu -q --timeout 180 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
  ok $rc || exit $rc
fi
if [[ $STEPS == *kbench* ]]; then
  for c in ${KB_CFGS:-c3}; do
    timeout -k 10 300 python tools/kernel_bench.py $c ${KB_ITERS:-200} >> gpurun_out/kbench.log 2>&1; rc=$?
    echo "kbench $c rc=$rc"; tail -1 gpurun_out/kbench.log
    ok $rc || exit $rc
  done
fi
if [[ $STEPS == *bench* && $STEPS != *kbench* ]] || [[ $STEPS == *,bench* ]]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
  ok $rc || exit $rc
fi
if [[ $STEPS == *prof* ]]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/prof.log 2>&1; rc=$?
  echo "prof rc=$rc"; tail -2 gpurun_out/prof.log
  find gpurun_out/prof -name "*stats*" | head
fi
exit 0
