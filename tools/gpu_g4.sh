cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g4 && export TMPDIR=/tmp
timeout -k 10 120 python3 tools/net_stamps.py c3 0,1,4096,4097 > gpurun_out/g4/stamps_c3.txt 2>&1 || exit 5
bash tools/kstats.sh g4c4 python3 tools/kernel_bench.py c4 50 > gpurun_out/g4/ks_c4.txt 2>&1 || exit 6
cat gpurun_out/g4/ks_c4.txt
