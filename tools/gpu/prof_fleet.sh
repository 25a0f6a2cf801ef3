# rocprofv3 kernel stats of the 28-tenant pod-server fleet (tools/podserver_once.py)
# and the x6 PMC passes.  usage (via gpurun): bash tools/gpu/prof_fleet.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-prof_fleet}
mkdir -p $O
timeout -k 10 200 python tools/podserver_once.py --tenants 28 --lanes 12 --window 6 > $O/once.json 2> $O/once.err || { echo once failed; tail -20 $O/once.err; exit 1; }
cat $O/once.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --tenants 28 --lanes 12 --window 4 > $O/prof.log 2>&1 || { echo prof failed; tail -10 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; rm -rf $O/prof
python3 - $O/kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:10]: print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'])
PY
bash tools/gpu/pmc_x6.sh ${1:-prof_fleet}_pmc
timeout -k 10 600 python bench.py --quota --json-out $O/quota.json 2>&1 | tee $O/quota.log || { echo quota failed; tail -30 $O/quota.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/quota.json'));print({k:d[k] for k in ('phase_a','phase_b','concurrent_tenants')})"
