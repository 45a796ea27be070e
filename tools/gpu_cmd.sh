timeout -k 10 200 python -u tools/lds_poison.py > gpurun_out/lp.log 2>&1; echo "rc=$?"; cat gpurun_out/lp.log | grep -v amdgpu.ids
T2="tests/test_hip_fullsize.py -q --timeout 180 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_hip_softlabels.py -k "not sharded" $T2 > gpurun_out/ta.log 2>&1; echo "softlabels(non-thread)+fullsize rc=$?"; grep -E "passed|failed|^FAILED" gpurun_out/ta.log | tail -6
