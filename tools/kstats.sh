# rocprofv3 kernel stats of a command: top kernels (name, calls, avg us, %)
#   bash tools/kstats.sh <tag> <command...>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$tag -o ks -- "$@" > gpurun_out/ks_$tag.log 2>&1 || { tail -5 gpurun_out/ks_$tag.log; exit 6; }
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/ks_$tag/ks_kernel_stats.csv')))[:${TOP:-10}]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1000,1), r['Percentage'])
"
