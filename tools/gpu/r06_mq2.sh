# Reserved-CU latency lanes, throughput lanes leaving latency requests to the
# priority lanes (lo_only): 16 throughput lanes over 8 masked queues, 2 / 4 / 8
# priority lanes on 16 / 32 reserved CUs, beside 20 YOLOS tenants.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_mq2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
run() {  # tag, podserver_once args...
  tag=$1; shift
  timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d.get('decode_token_latency_ms'), {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/$tag.json $tag
}
M="--mix yolos:20,llama-dec:8 --window 8"
run pl4_cus16 $M --priority-lanes 4 --latency-cus 16 --masked-queues 8 || exit 1
run pl2_cus16 $M --priority-lanes 2 --latency-cus 16 --masked-queues 8 || exit 1
run pl4_cus32 $M --priority-lanes 4 --latency-cus 32 --masked-queues 8 || exit 1
run pl8_cus32 $M --priority-lanes 8 --latency-cus 32 --masked-queues 6 || exit 1
run pl4_cus32_mq4 $M --priority-lanes 4 --latency-cus 32 --masked-queues 4 || exit 1
run base $M || exit 1
