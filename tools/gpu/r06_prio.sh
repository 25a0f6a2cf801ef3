# Latency lanes A/B (mixed YOLOS + decode fleet, and the plain YOLOS fleet), the
# fuzz + decode GPU tests, then the 7-pod CU-mask PMC.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_prio; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_program_fuzz_gpu.py tests/test_decode_gpu.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed|Falsifying" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for pl in 0 2; do
    timeout -k 10 300 python3 tools/podserver_once.py --mix yolos:20,llama-dec:8 --window 8 --priority-lanes $pl > $O/mix_pl${pl}_r$r.json 2> $O/mix_pl${pl}_r$r.err || { echo "mix $pl failed"; tail -5 $O/mix_pl${pl}_r$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('mix pl', sys.argv[2], d['inf_per_s'], d['decode_token_latency_ms'], {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/mix_pl${pl}_r$r.json $pl
  done
done
for pl in 0 2; do
  timeout -k 10 300 python3 tools/podserver_once.py --tenants 28 --window 8 --priority-lanes $pl > $O/yolos_pl$pl.json 2> $O/yolos_pl$pl.err || { echo "yolos $pl failed"; tail -5 $O/yolos_pl$pl.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('yolos pl', sys.argv[2], d['inf_per_s'], d['sclk_mhz'])" $O/yolos_pl$pl.json $pl
done
bash tools/gpu/cumask_pmc7.sh r06_prio/cumask7
