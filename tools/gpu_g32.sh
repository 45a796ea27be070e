#!/bin/bash
# LeNet d/du tangent kernel with prefetch and no plane clearing: LeNet tests,
# HVP kernel stats and timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
mkdir -p gpurun_out/g32
timeout -k 10 600 python -u -m pytest tests/test_hip_lenet.py tests/test_hip_lenet_c5.py tests/test_hip_lds_poison.py tests/test_hip_variants.py -x -q --timeout 300 --timeout-method thread > gpurun_out/g32/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/g32/pytest.log; [ $rc -eq 0 ] || exit $rc
TOP=6 bash tools/kstats.sh g32 python3 tools/lenet_probe.py --T 1 --reps 1 --hvp 3 > gpurun_out/g32/ks.txt 2>&1 || exit 6
cat gpurun_out/g32/ks.txt
timeout -k 10 300 python3 tools/lenet_probe.py --T 2 --reps 1 --hvp 5 > gpurun_out/g32/probe.txt 2>&1 || exit 7
grep -v amdgpu gpurun_out/g32/probe.txt
exit 0
