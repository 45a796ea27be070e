cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
for i in 1 2; do
  echo "old:"; PSVI_LIB_AB=$GRAFT_REPO_ROOT/blackbox-coresets-vi_amd/psvi/runtime/libpsvi_hip_ab.so timeout -k 10 200 python3 tools/stream_cost_sweep.py 100:150 2>&1 | grep first || exit 3
  echo "new:"; timeout -k 10 200 python3 tools/stream_cost_sweep.py 100:150 2>&1 | grep first || exit 4
done
