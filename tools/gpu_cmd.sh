set -o pipefail
timeout -k 10 120 python -u tools/ks_stamps.py 8 0 1024 > gpurun_out/ks.log 2>&1 && cat gpurun_out/ks.log &&
timeout -k 10 120 python -u tools/ks_stamps.py 8 0 1024 256 > gpurun_out/ks256.log 2>&1 && head -n 9 gpurun_out/ks256.log &&
timeout -k 10 120 python -u tools/ks_stamps.py 1 0 1024 > gpurun_out/ks1.log 2>&1 && cat gpurun_out/ks1.log &&
timeout -k 10 120 python -u tools/net_stamps.py c3 0 1 0 > gpurun_out/ns1.log 2>&1 && cat gpurun_out/ns1.log &&
timeout -k 10 120 python -u tools/net_stamps.py c3 0 8 0 > gpurun_out/ns8.log 2>&1 && cat gpurun_out/ns8.log &&
timeout -k 10 120 python -u tools/net_stamps.py c4 0 8 0 > gpurun_out/ns8c4.log 2>&1 && cat gpurun_out/ns8c4.log
