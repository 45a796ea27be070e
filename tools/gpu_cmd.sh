set -o pipefail
export PYTHONPATH=$PWD/blackbox-coresets-vi_amd:$PWD/oracle:$PWD/tests:$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -3 gpurun_out/pytest_gpu.log && \
timeout -k 10 200 python -u tools/loop_overhead.py > gpurun_out/loop_ovh2.log 2>&1 && cat gpurun_out/loop_ovh2.log && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv.json 2> gpurun_out/bench_drv.err && tail -c 300 gpurun_out/bench_drv.json
