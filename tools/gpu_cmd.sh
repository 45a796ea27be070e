T2="tests/test_hip_fullsize.py -q --timeout 180 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_hip_softlabels.py -k "not sharded" $T2 > gpurun_out/ta.log 2>&1; echo "softlabels(non-thread)+fullsize rc=$?"; grep -E "passed|failed|^FAILED" gpurun_out/ta.log | tail -6
ROUND=r04 bash tools/round_session.sh
