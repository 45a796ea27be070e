#!/bin/bash
# Round-6 closing evidence after the paired HVP sample and the nt state loads:
# GPU suite, smoke, bench, bench kernel stats; hyper_step timing and kernel
# stats; C3 psvi_hvp timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
STEPS=tests,smoke,bench,prof EXTRA=none bash tools/round6_session.sh || exit $?
mkdir -p gpurun_out/g30
timeout -k 10 200 python3 tools/hyper_probe.py 3 hyper > gpurun_out/g30/hyper.txt 2>&1 || { tail -5 gpurun_out/g30/hyper.txt; exit 4; }
cat gpurun_out/g30/hyper.txt
timeout -k 10 120 python3 tools/hvp_probe.py --cfg c3 --n 200 > gpurun_out/g30/hvp.txt 2>&1 || { tail -5 gpurun_out/g30/hvp.txt; exit 5; }
cat gpurun_out/g30/hvp.txt
bash tools/kstats.sh g30h python3 tools/hyper_probe.py 2 hyper > gpurun_out/g30/ks.txt 2>&1 || exit 6
cat gpurun_out/g30/ks.txt
exit 0
