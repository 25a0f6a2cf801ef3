set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5_bf16prof; mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --tenants 28 --window 4 --dtype bf16 > $O/prof.log 2>&1 || { echo prof failed; tail -10 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; rm -rf $O/prof
python3 - $O/kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]: print(r['Name'][:110], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'])
PY
