cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g10 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_hip_stream_bf.py tests/test_hip_cg.py tests/test_hip_net_geo.py tests/test_hip_sharded_run.py tests/test_hip_parity.py tests/test_bench_shared_gpu.py tests/test_hip_hypergrad.py tests/test_hip_sharded_trainer.py tests/test_hip_variants.py tests/test_run_psvi_gpu.py tests/test_hip_hvp.py tests/test_hip_evaluate.py tests/test_hip_lds_poison.py tests/test_isa_hazards.py > gpurun_out/g10/t.log 2>&1 || { tail -30 gpurun_out/g10/t.log; exit 3; }
tail -2 gpurun_out/g10/t.log; grep -E "rel l2" gpurun_out/g10/t.log | head
timeout -k 10 200 python3 tools/hyper_probe.py 3 hyper > gpurun_out/g10/hyper.txt 2>&1 || { tail -5 gpurun_out/g10/hyper.txt; exit 4; }
cat gpurun_out/g10/hyper.txt
timeout -k 10 120 python3 tools/hvp_probe.py --cfg c3 > gpurun_out/g10/hvp.txt 2>&1 || { tail -5 gpurun_out/g10/hvp.txt; exit 5; }
cat gpurun_out/g10/hvp.txt
bash tools/kstats.sh g10h python3 tools/hyper_probe.py 2 hyper > gpurun_out/g10/ks.txt 2>&1 || exit 6
cat gpurun_out/g10/ks.txt
timeout -k 10 300 python3 tools/overlap_timing.py --world 8 --rank 0 --delays 0,10,20,40 --T 30 > gpurun_out/g10/overlap.jsonl 2>&1 || { tail -5 gpurun_out/g10/overlap.jsonl; exit 7; }
cat gpurun_out/g10/overlap.jsonl
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-lenet --no-c2 > gpurun_out/g10/bench.json 2> gpurun_out/g10/bench.err || { tail -5 gpurun_out/g10/bench.err; exit 8; }
cat gpurun_out/g10/bench.json
