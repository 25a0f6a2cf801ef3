# Decode kernels after the argmax / decode-attention staging fixes: GPU tests,
# decode rates alone and beside YOLOS, and 8 decoders' kernel stats.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_dec2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
for mix in llama-dec:1 llama-dec:8 yolos:20,llama-dec:8; do
  tag=$(echo $mix | tr ':,' '__')
  timeout -k 10 300 python3 tools/podserver_once.py --mix $mix --window 8 > $O/$tag.json 2> $O/$tag.err || { echo "$mix failed"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d['decode_token_latency_ms'], {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/$tag.json $mix
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --mix llama-dec:8 --window 4 > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/dec8_kernel_stats.csv; rm -rf $O/prof
python3 - $O/dec8_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(f'{100*float(r["TotalDurationNs"])/tot:5.1f}% {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:8.1f}us {r["Name"][:90]}')
PY
