cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g21 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_hip_stream_bf.py tests/test_hip_parity.py tests/test_hip_loop_resident.py tests/test_hip_fullsize.py > gpurun_out/g21/t.log 2>&1 || { tail -30 gpurun_out/g21/t.log; exit 3; }
tail -1 gpurun_out/g21/t.log
timeout -k 10 300 python3 tools/stream_cost_sweep.py 100:150 > gpurun_out/g21/sweep.txt 2>&1 || exit 4
tail -1 gpurun_out/g21/sweep.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-lenet --no-c2 --no-trainers --no-c4 > gpurun_out/g21/bench.json 2>/dev/null || exit 8
python3 -c "import json; d=json.loads(open('gpurun_out/g21/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernels'])"
