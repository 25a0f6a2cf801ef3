# The server's generate loop (decode steps replayed back to back, ids fed back
# on the device, one request per K tokens): GPU tests, decode rates at
# K = 1 / 16 / 64, 8 decoders and the YOLOS mix at K = 16.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_genloop; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_decode_tenants.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
run() {  # tag, podserver_once args...
  tag=$1; shift
  timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d.get('decode_token_latency_ms'), {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/$tag.json $tag
}
run dec1_k1 --mix llama-dec:1 --window 8 || exit 1
run dec1_k16 --mix llama-dec:1 --window 8 --gen-chunk 16 || exit 1
run dec1_k64 --mix llama-dec:1 --window 8 --gen-chunk 64 || exit 1
run dec8_k16 --mix llama-dec:8 --window 8 --gen-chunk 16 || exit 1
run mix_k16 --mix yolos:20,llama-dec:8 --window 8 --gen-chunk 16 || exit 1
