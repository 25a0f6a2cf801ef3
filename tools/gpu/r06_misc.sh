# Strided unary / host-copy tests, the fleet's kernel stats (no per-inference
# at::native copy left), then the h3 attention waves A/B (8 vs 4) and a bf16 fleet.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_misc; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tenant_ops_gpu.py tests/test_tenant_programs_gpu.py tests/test_podserver_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --tenants 28 --window 4 > $O/prof.log 2>&1 || { echo prof failed; tail -10 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; rm -rf $O/prof
python3 - $O/kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:9]: print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'])
PY
one() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python3 tools/podserver_once.py --tenants 28 --window 10 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d['sclk_mhz'], round(d['inf_per_s']/d['sclk_mhz'],4))" $O/$tag.json $tag
}
for r in 1 2; do
  one w8_r$r --h3-attn-waves 8 || exit 1
  one w4_r$r --h3-attn-waves 4 || exit 1
done
one bf16 --dtype bf16 || exit 1
