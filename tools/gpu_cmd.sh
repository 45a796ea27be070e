set -o pipefail
export PYTHONPATH=$PWD/blackbox-coresets-vi_amd:$PWD/oracle:$PWD/tests:$PWD
timeout -k 10 600 python -u bench.py > gpurun_out/bench_def.json 2> gpurun_out/bench_def.err && tail -c 400 gpurun_out/bench_def.json
