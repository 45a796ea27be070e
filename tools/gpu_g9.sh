cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g9 && export TMPDIR=/tmp
timeout -k 10 120 python3 tools/net_time_probe.py c3 0,16 > gpurun_out/g9/ntp.txt 2>&1 || exit 5
timeout -k 10 120 python3 tools/net_time_probe.py c3 0,16 --draw >> gpurun_out/g9/ntp.txt 2>&1 || exit 5
cat gpurun_out/g9/ntp.txt
timeout -k 10 300 python3 tools/rank_timing.py --cfg c4 --world 8 --schedule run --iters 40 > gpurun_out/g9/rank_w8_run.jsonl 2> gpurun_out/g9/rank.err || { tail -5 gpurun_out/g9/rank.err; exit 6; }
tail -3 gpurun_out/g9/rank_w8_run.jsonl
