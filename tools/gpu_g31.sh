#!/bin/bash
# LeNet (C5) HVP kernel stats: where the 18 ms go.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
mkdir -p gpurun_out/g31
TOP=16 bash tools/kstats.sh g31 python3 tools/lenet_probe.py --T 1 --reps 1 --hvp 3 > gpurun_out/g31/ks.txt 2>&1 || exit 6
cat gpurun_out/g31/ks.txt
exit 0
