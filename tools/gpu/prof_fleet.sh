# rocprofv3 kernel stats of the 28-tenant pod-server fleet (tools/podserver_once.py).
# usage (via gpurun): bash tools/gpu/prof_fleet.sh <tag> [fp32|bf16]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-prof_fleet}; DT=${2:-fp32}; mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --tenants 28 --window 4 --dtype $DT > $O/prof.log 2>&1 || { echo prof failed; tail -10 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_$DT.csv; rm -rf $O/prof
python3 - $O/kernel_stats_$DT.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]: print(r['Name'][:110], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'])
PY
