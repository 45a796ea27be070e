set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && tail -c 3000 gpurun_out/bench.json &&
timeout -k 10 200 python -u tools/rank_timing.py --cfg c4 --world 8 --iters 50 > gpurun_out/rt_c4.log 2>&1 && tail -n 12 gpurun_out/rt_c4.log &&
timeout -k 10 200 python -u tools/rank_timing.py --cfg weak --world 8 --iters 50 > gpurun_out/rt_weak.log 2>&1 && tail -n 3 gpurun_out/rt_weak.log &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rt -o rt -- python tools/rank_timing.py --cfg c4 --world 8 --ranks 0,7 --iters 30 > gpurun_out/prof_rt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b -o b -- python bench.py --steps 200 > gpurun_out/prof_b.log 2>&1 && echo PROF_OK
