# Full GPU check of the committed tree (the driver's round-end steps): pytest -m gpu, smoke(), the default
# bench.py (the driver's command), then fleet kernel stats.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-full_check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo gpu tests failed; grep -E "FAILED|Error|assert" $O/gputests.log | head -30; tail -5 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python3 -c "import json;d=json.load(open('$O/bench.json'));print({k:d.get(k) for k in ('value','aggregate_inf_per_s','matrix_pipe_util_pct','aggregate_vs_single_pod','bf16_fleet_inf_per_s','rank0_sclk_mhz')})"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --tenants 28 --window 4 > $O/prof.log 2>&1 || { echo prof failed; tail -10 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; rm -rf $O/prof
python3 - $O/kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]: print(r['Name'][:100], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'])
PY
