cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g12 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_hip_sharded_run.py > gpurun_out/g12/t.log 2>&1 || { tail -30 gpurun_out/g12/t.log; exit 3; }
tail -2 gpurun_out/g12/t.log
timeout -k 10 300 python3 tools/overlap_timing.py --world 8 --rank 0 --delays 0,10,20,40 --T 30 > gpurun_out/g12/overlap.jsonl 2>&1 || { tail -5 gpurun_out/g12/overlap.jsonl; exit 7; }
cat gpurun_out/g12/overlap.jsonl
timeout -k 10 300 python3 tools/overlap_timing.py --world 2 --rank 0 --delays 0,20 --T 30 > gpurun_out/g12/overlap_w2.jsonl 2>&1 || { tail -5 gpurun_out/g12/overlap_w2.jsonl; exit 8; }
cat gpurun_out/g12/overlap_w2.jsonl
