set -o pipefail
export PYTHONPATH=$PWD/blackbox-coresets-vi_amd:$PWD/oracle:$PWD/tests:$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_parity.py -k net_draw > gpurun_out/t_draw2.log 2>&1; rc=$?; tail -15 gpurun_out/t_draw2.log; exit $rc
