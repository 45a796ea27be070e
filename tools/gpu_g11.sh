cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g11 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_hip_stream_bf.py tests/test_hip_cg.py tests/test_hip_hvp.py tests/test_hip_hypergrad.py tests/test_hip_loop_resident.py tests/test_hip_parity.py > gpurun_out/g11/t.log 2>&1 || { tail -30 gpurun_out/g11/t.log; exit 3; }
tail -2 gpurun_out/g11/t.log
timeout -k 10 200 python3 tools/hyper_probe.py 3 hyper > gpurun_out/g11/hyper.txt 2>&1 || { tail -5 gpurun_out/g11/hyper.txt; exit 4; }
cat gpurun_out/g11/hyper.txt
bash tools/kstats.sh g11h python3 tools/hyper_probe.py 2 hyper > gpurun_out/g11/ks.txt 2>&1 || exit 6
head -12 gpurun_out/g11/ks.txt
timeout -k 10 300 python3 tools/overlap_timing.py --world 8 --rank 0 --delays 0,10,20,40 --T 30 > gpurun_out/g11/overlap.jsonl 2>&1 || { tail -5 gpurun_out/g11/overlap.jsonl; exit 7; }
cat gpurun_out/g11/overlap.jsonl
bash tools/kstats.sh g11b python3 bench.py --no-cpu-baseline --no-lenet --no-c2 --no-trainers > gpurun_out/g11/ksb.txt 2>&1 || exit 8
head -8 gpurun_out/g11/ksb.txt
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-lenet --no-c2 > gpurun_out/g11/bench.json 2> gpurun_out/g11/bench.err || { tail -5 gpurun_out/g11/bench.err; exit 9; }
cat gpurun_out/g11/bench.json
