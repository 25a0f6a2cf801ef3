# Pinned staging for the pod server's per-request copies (input H2D in-stream,
# outputs + counters D2H behind one synchronisation): GPU tests, decode rates,
# the mix, a bench; then reserved-CU latency lanes with fewer throughput lanes
# (does the number of CU-masked queues starve the decoders?).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_pinned; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_podserver_gpu.py tests/test_tenant_ops_gpu.py tests/test_training_fuzz_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
run() {  # tag, podserver_once args...
  tag=$1; shift
  timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d.get('decode_token_latency_ms'), {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/$tag.json $tag
}
run dec1 --mix llama-dec:1 --window 8 || exit 1
run dec8 --mix llama-dec:8 --window 8 || exit 1
run mix --mix yolos:20,llama-dec:8 --window 8 || exit 1
run yolos28 --mix yolos:28 --window 8 || exit 1
run mix_cus16_l4 --mix yolos:20,llama-dec:8 --window 8 --priority-lanes 2 --latency-cus 16 --lanes 4 || exit 1
run mix_pl2_l4 --mix yolos:20,llama-dec:8 --window 8 --priority-lanes 2 --lanes 4 || exit 1
run mix_cus16_l8 --mix yolos:20,llama-dec:8 --window 8 --priority-lanes 2 --latency-cus 16 --lanes 8 || exit 1
