cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_stream.py tests/test_hip_parity.py tests/test_hip_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_stream.log 2>&1; rc=$?
tail -25 gpurun_out/pt_stream.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --no-trainers --no-lenet --steps 300 --warmup 20 > gpurun_out/bench_stream.log 2>&1; rc=$?; tail -1 gpurun_out/bench_stream.log | cut -c1-600; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stream -o bench -- python3 bench.py --no-cpu-baseline --no-trainers --no-lenet --steps 200 --warmup 20 > gpurun_out/prof_stream.log 2>&1; echo prof rc=$?
