cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g14 && export TMPDIR=/tmp
for abl in 0 1 2 4 7 48 55; do
  timeout -k 10 120 python3 tools/lenet_probe.py --abl $abl --T 5 --reps 2 > gpurun_out/g14/abl_$abl.txt 2>&1 || { tail -5 gpurun_out/g14/abl_$abl.txt; exit 3; }
  echo "abl $abl: $(grep -v amdgpu gpurun_out/g14/abl_$abl.txt | tail -1)"
done
