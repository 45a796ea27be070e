cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g16 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_hip_stream_bf.py > gpurun_out/g16/t.log 2>&1 || { tail -30 gpurun_out/g16/t.log; exit 3; }
tail -1 gpurun_out/g16/t.log
timeout -k 10 120 python3 tools/bf_stamps.py > gpurun_out/g16/bf.txt 2>&1 || { tail -5 gpurun_out/g16/bf.txt; exit 4; }
tail -4 gpurun_out/g16/bf.txt
bash tools/kstats.sh g16 python3 bench.py --no-cpu-baseline --no-lenet --no-c2 --no-trainers --no-c4 --steps 200 --warmup 20 > gpurun_out/g16/ks.txt 2>&1 || exit 6
head -3 gpurun_out/g16/ks.txt
tail -1 gpurun_out/ks_g16.log | cut -c1-200
