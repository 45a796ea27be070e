cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g2 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_loop_resident.py tests/test_hip_stream_bf.py > gpurun_out/g2/t.log 2>&1 || { tail -30 gpurun_out/g2/t.log; exit 3; }
tail -3 gpurun_out/g2/t.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-lenet --no-trainers > gpurun_out/g2/b.json 2> gpurun_out/g2/b.err || { tail -20 gpurun_out/g2/b.err; exit 4; }
cat gpurun_out/g2/b.json
