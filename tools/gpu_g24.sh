cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g24 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_hip_lenet.py tests/test_hip_lenet_c5.py tests/test_hip_variants.py tests/test_hip_softlabels.py tests/test_hip_hvp.py tests/test_hip_evaluate.py > gpurun_out/g24/t.log 2>&1 || { tail -30 gpurun_out/g24/t.log; exit 3; }
tail -1 gpurun_out/g24/t.log
timeout -k 10 200 python3 tools/lenet_probe.py --T 5 --reps 2 --hvp 3 > gpurun_out/g24/probe.txt 2>&1 || { tail -5 gpurun_out/g24/probe.txt; exit 4; }
grep -v amdgpu gpurun_out/g24/probe.txt
TOP=6 bash tools/kstats.sh g24 python3 tools/lenet_probe.py --T 3 --reps 1 > gpurun_out/g24/ks.txt 2>&1 || exit 5
cat gpurun_out/g24/ks.txt
