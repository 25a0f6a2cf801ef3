# Round 5: the LN plane handoff (nos_gemm_f32h3_ln_out) -- tests, fleet A/B
# (handoff on vs off, twice), rocprofv3 kernel stats of the 28-tenant fleet,
# and the mixed-family fleet (YOLOS + ResNet-18 + Llama) profile.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_handoff
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ln_handoff_gpu.py tests/test_tenant_programs_gpu.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
CONFIGS="on1: off1:NOS_AMD_LN_HANDOFF=off on2: off2:NOS_AMD_LN_HANDOFF=off" bash tools/gpu/ab_fleet_env.sh || exit 1
cp gpurun_out/fleet_ab/results.txt $O/ab.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --tenants 28 --window 4 > $O/prof.log 2>&1 || { echo prof failed; tail -10 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; rm -rf $O/prof
python3 - $O/kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'])
PY
timeout -k 10 400 python tools/podserver_once.py --mix yolos:16,resnet:6,llama:6 --window 8 > $O/mix.json 2> $O/mix.err || { echo mix failed; tail -20 $O/mix.err; exit 1; }
cat $O/mix.json
