# Round 5: LayerNorm in the LN-GEMM's A load (nos_gemm_f32h3_lna) from the
# residual GEMM's row statistics (nos_gemm_f32h3_stats) -- tests, then the
# 28-tenant fleet with the hand-off on vs off (twice), then kernel stats.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5_lna}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v tests/test_ln_handoff_gpu.py tests/test_gemm_h3_gpu.py --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -3 $O/tests.log
CONFIGS="on1:NOS_AMD_LN_HANDOFF=on off1: on2:NOS_AMD_LN_HANDOFF=on off2:" bash tools/gpu/ab_fleet_env.sh || exit 1
cp gpurun_out/fleet_ab/results.txt $O/ab.txt
cd /tmp && NOS_AMD_LN_HANDOFF=on timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --tenants 28 --lanes 12 --window 4 > $O/prof.log 2>&1 || { echo prof failed; tail -10 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; rm -rf $O/prof
python3 - $O/kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]: print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'])
PY
