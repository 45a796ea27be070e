cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g17 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_hip_stream_bf.py tests/test_hip_loop_resident.py tests/test_hip_parity.py > gpurun_out/g17/t.log 2>&1 || { tail -30 gpurun_out/g17/t.log; exit 3; }
tail -1 gpurun_out/g17/t.log
bash tools/kstats.sh g17 python3 bench.py --no-cpu-baseline --no-lenet --no-c2 --no-trainers --no-c4 --steps 200 --warmup 20 > gpurun_out/g17/ks.txt 2>&1 || exit 6
head -3 gpurun_out/g17/ks.txt
