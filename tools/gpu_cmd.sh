set -o pipefail
export PYTHONPATH=$PWD/blackbox-coresets-vi_amd:$PWD/oracle:$PWD/tests:$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_parity.py tests/test_bench_shared_gpu.py tests/test_hip_sharded_trainer.py tests/test_hip_fullsize.py > gpurun_out/t_draw.log 2>&1 && tail -3 gpurun_out/t_draw.log && \
timeout -k 10 200 python -u tools/rank_timing.py --cfg c4 --world 8 --schedule run --iters 50 > gpurun_out/rt_run_c4.log 2>&1 && tail -1 gpurun_out/rt_run_c4.log && \
timeout -k 10 200 python -u tools/rank_timing.py --cfg c4 --world 8 --iters 50 > gpurun_out/rt_ph_c4.log 2>&1 && tail -1 gpurun_out/rt_ph_c4.log && \
timeout -k 10 200 python -u tools/rank_timing.py --cfg weak --world 8 --schedule run --iters 50 > gpurun_out/rt_run_weak.log 2>&1 && tail -1 gpurun_out/rt_run_weak.log && \
timeout -k 10 200 python -u tools/loop_overhead.py > gpurun_out/loop_ovh.log 2>&1 && cat gpurun_out/loop_ovh.log
