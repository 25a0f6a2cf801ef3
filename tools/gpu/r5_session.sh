# Round-5 evidence pass (GPU box, via gpurun): the tenant-program GPU tests,
# BASELINE config 5 composed (real pod server + trainer pod), h3 PMC passes
# (GEMM / LN split / attention VALU per MFMA) and fleet kernel stats.
# usage: bash tools/gpu/r5_session.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5_session}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tenant_programs_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 900 python bench.py --quota --composed --json-out $O/composed.json > $O/composed.log 2>&1 || { echo composed failed; tail -30 $O/composed.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/composed.json'));print({k:d[k] for k in d if k.startswith('phase') or k in ('quota_vs_footprint','repartition')})"
bash tools/gpu/pmc_h3.sh ${1:-r5_session}/pmc || exit 1
cd $R
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --tenants 28 --lanes 12 --window 4 > $O/prof.log 2>&1 || { echo prof failed; tail -10 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; rm -rf $O/prof
python3 - $O/kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:10]: print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'])
PY
