cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g3 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_net_geo.py tests/test_hip_net_lds.py tests/test_hip_net_mloop.py > gpurun_out/g3/t.log 2>&1 || { tail -30 gpurun_out/g3/t.log; exit 3; }
tail -3 gpurun_out/g3/t.log
timeout -k 10 120 python3 tools/net_stamps.py c3 0 > gpurun_out/g3/stamps_c3.txt 2>&1 || exit 5
timeout -k 10 120 python3 tools/net_stamps.py c4 0 > gpurun_out/g3/stamps_c4.txt 2>&1 || exit 5
bash tools/kstats.sh g3k python3 tools/kernel_bench.py c3 200 > gpurun_out/g3/ks_c3.txt 2>&1 || exit 6
cat gpurun_out/g3/ks_c3.txt
