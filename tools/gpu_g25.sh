#!/bin/bash
# A/B of the streaming kernel's tiled-state load cache policy (builds
# libpsvi_hip_aux<A>.so with -DPSVI_STATE_LOAD_AUX=A): C3 loop timing and the
# kernel's FETCH_SIZE / WRITE_SIZE per variant.  The box's tree is a scratch
# copy, so each variant is copied over libpsvi_hip.so in turn.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
R=blackbox-coresets-vi_amd/psvi/runtime
cp $R/libpsvi_hip.so $R/libpsvi_hip_aux0.so
mkdir -p gpurun_out/ab
CMD="python3 bench.py --no-cpu-baseline --no-trainers --no-lenet --no-c4 --no-c2 --steps 50 --warmup 5"
for A in ${VARIANTS:-0 2 18}; do
  cp $R/libpsvi_hip_aux$A.so $R/libpsvi_hip.so
  echo "aux $A"
  timeout -k 10 200 python3 tools/stream_cost_sweep.py 100:150 2>&1 | grep first || exit 3
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/ab/a$A/p$c -o p -- $CMD > gpurun_out/ab/a${A}_$c.log 2>&1 || exit 4
  done
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/a$A/trace -o trace -- $CMD > gpurun_out/ab/a${A}_trace.log 2>&1 || exit 5
  python3 tools/pmc_report.py gpurun_out/ab/a$A 2>&1 | grep -A4 "stream_bf2" | head -12
done
exit 0
