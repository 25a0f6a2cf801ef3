# Decode latency beside a YOLOS fleet: one-queue dispatch without priority
# lanes, with 2 priority lanes, and with 16 / 32 CUs reserved for them; then
# the GPU decode tests (incl. generation with reserved CUs).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_lat; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
for cfg in "0 0" "2 0" "2 16" "2 32"; do
  set -- $cfg
  tag=pl$1_cu$2
  timeout -k 10 300 python3 tools/podserver_once.py --mix yolos:20,llama-dec:8 --window 8 --priority-lanes $1 --latency-cus $2 > $O/mix_$tag.json 2> $O/mix_$tag.err || { echo "mix $tag failed"; tail -5 $O/mix_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('mix', sys.argv[2], d['inf_per_s'], d['decode_token_latency_ms'], {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/mix_$tag.json $tag
done
