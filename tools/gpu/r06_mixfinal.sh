# The last tree beside the YOLOS fleet: 20 YOLOS + 8 decoders with the generate loop
# (16 tokens per request), on the default server and with 8 priority lanes on 32
# reserved CUs; a request per token for comparison.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_mixfinal; mkdir -p $O
run() {  # tag, podserver_once args...
  tag=$1; shift
  timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d.get('decode_token_latency_ms'), {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/$tag.json $tag
}
M="--mix yolos:20,llama-dec:8 --window 8"
run k1 $M || exit 1
run k16 $M --gen-chunk 16 || exit 1
run k16_cus32_pl8 $M --gen-chunk 16 --priority-lanes 8 --latency-cus 32 --masked-queues 6 || exit 1
run dec1_k64 --mix llama-dec:1 --window 8 --gen-chunk 64 || exit 1
run dec8_k16 --mix llama-dec:8 --window 8 --gen-chunk 16 || exit 1
