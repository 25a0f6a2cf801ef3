# Training step kernel stats after the log-sum-exp loss, the latency-lane A/B
# on the one-queue dispatcher, then BASELINE config 5 composed (shared and split).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_main2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train_ops_gpu.py tests/test_training_tenants_gpu.py -q --timeout 300 --timeout-method thread > $O/train_tests.log 2>&1 || { echo train tests failed; grep -E "Error|assert|FAILED|failed" $O/train_tests.log | head -30; exit 1; }
tail -1 $O/train_tests.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trainprof -o run -- python3 $R/tools/train_once.py --seq 2048 --steps 3 --small 1) > $O/trainprof.log 2>&1 || { echo trainprof failed; tail -5 $O/trainprof.log; exit 1; }
grep -h '^{' $O/trainprof.log || true
python3 - $O <<'PY'
import csv, glob, sys
o = sys.argv[1]
f = glob.glob(f"{o}/trainprof/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(f'{100*float(r["TotalDurationNs"])/tot:5.1f}% {int(r["Calls"]):6d} {r["Name"][:110]}')
bad = [r["Name"][:90] for r in rows if any(s in r["Name"] for s in ("Cijk", "hipblaslt", "softmax_warp", "SoftMax"))]
print("library GEMM / softmax kernels:", bad if bad else "none")
PY
for pl in 0 2; do
  timeout -k 10 300 python3 tools/podserver_once.py --mix yolos:20,llama-dec:8 --window 8 --priority-lanes $pl > $O/mix_pl$pl.json 2> $O/mix_pl$pl.err || { echo "mix $pl failed"; tail -5 $O/mix_pl$pl.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('mix pl', sys.argv[2], d['inf_per_s'], d['decode_token_latency_ms'], {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/mix_pl$pl.json $pl
done
bash tools/gpu/r06_config5.sh
