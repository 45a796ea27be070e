cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g6 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_net_geo.py tests/test_hip_net_lds.py tests/test_hip_net_mloop.py tests/test_hip_parity.py tests/test_hip_stream_bf.py tests/test_hip_stream.py tests/test_hip_lds_poison.py > gpurun_out/g6/t.log 2>&1 || { tail -30 gpurun_out/g6/t.log; exit 3; }
tail -2 gpurun_out/g6/t.log
timeout -k 10 120 python3 tools/net_stamps.py c3 0,1 > gpurun_out/g6/stamps_c3.txt 2>&1 || exit 5
timeout -k 10 120 python3 tools/net_stamps.py c4 0 > gpurun_out/g6/stamps_c4.txt 2>&1 || exit 5
bash tools/kstats.sh g6 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lenet --no-trainers --no-c2 > gpurun_out/g6/ks.txt 2>&1 || exit 6
cat gpurun_out/g6/ks.txt; grep -h '"value"' gpurun_out/ks_g6.log | cut -c1-300
