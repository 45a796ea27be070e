cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g15 && export TMPDIR=/tmp
TOP=14 bash tools/kstats.sh g15 python3 tools/rank_timing.py --cfg c4 --world 8 --ranks 0 --schedule run --iters 40 > gpurun_out/g15/ks.txt 2>&1 || { cat gpurun_out/g15/ks.txt; exit 6; }
cat gpurun_out/g15/ks.txt
