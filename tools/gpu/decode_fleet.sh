# Decode tenants on the pod server: one alone, 8 together, and a YOLOS + decode
# fleet (per-token latency, tokens/s), then kernel stats of the mixed fleet.
# usage (GPU box, repo root): bash tools/gpu/decode_fleet.sh <tag> [mix]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-decode_fleet}; MIX=${2:-yolos:20,llama-dec:8}; mkdir -p $O
for m in llama-dec:1 llama-dec:8 $MIX; do
  timeout -k 10 300 python3 tools/podserver_once.py --mix $m --window 8 > $O/run_${m//[:,]/_}.json 2> $O/run_${m//[:,]/_}.err || { echo "$m failed"; tail -5 $O/run_${m//[:,]/_}.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d['decode_token_latency_ms'], {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/run_${m//[:,]/_}.json $m
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --mix $MIX --window 4 > $O/prof.log 2>&1 || { echo prof failed; tail -10 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; rm -rf $O/prof
python3 - $O/kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]: print(r['Name'][:100], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'])
PY
