set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_hip_kstream.py tests/test_hip_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -n 3 gpurun_out/tk.log; [ $rc = 0 ] &&
timeout -k 10 120 python -u tools/ks_stamps.py 8 0 1024 > gpurun_out/ks.log 2>&1 && tail -n 8 gpurun_out/ks.log &&
timeout -k 10 120 python -u tools/ks_stamps.py 1 0 1024 > gpurun_out/ks1.log 2>&1 && tail -n 8 gpurun_out/ks1.log
