cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/t2.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/rank_timing.py --cfg c4 --world 8 > gpurun_out/rt_c4.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/rank_timing.py --cfg weak --world 8 > gpurun_out/rt_weak.log 2>&1 || exit $?
tail -3 gpurun_out/rt_c4.log gpurun_out/rt_weak.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-trainers --no-lenet > gpurun_out/b1.log 2>&1; echo bench rc=$?; tail -c 1500 gpurun_out/b1.log
