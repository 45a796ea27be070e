cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g18 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_hip_stream_bf.py tests/test_hip_kstream.py tests/test_hip_sharded_run.py tests/test_hip_fullsize.py tests/test_hip_parity.py tests/test_hip_loop_resident.py > gpurun_out/g18/t.log 2>&1 || { tail -30 gpurun_out/g18/t.log; exit 3; }
tail -1 gpurun_out/g18/t.log
timeout -k 10 300 python3 tools/rank_timing.py --cfg c4 --world 8 --schedule run > gpurun_out/g18/rank.jsonl 2>&1 || { tail -5 gpurun_out/g18/rank.jsonl; exit 6; }
tail -1 gpurun_out/g18/rank.jsonl
TOP=8 bash tools/kstats.sh g18 python3 tools/rank_timing.py --cfg c4 --world 8 --ranks 0 --schedule run --iters 40 > gpurun_out/g18/ks.txt 2>&1 || exit 7
cat gpurun_out/g18/ks.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-lenet --no-c2 --no-trainers --steps 200 --warmup 20 > gpurun_out/g18/bench.json 2>/dev/null || exit 8
python3 -c "import json; d=json.loads(open('gpurun_out/g18/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['c4_1gpu'])"
