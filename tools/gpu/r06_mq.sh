# Reserved-CU latency lanes with the throughput lanes sharing a bounded number
# of CU-masked streams (each one a hardware queue): 16 lanes over 8 / 4 / 12
# masked queues, 16 and 32 reserved CUs, beside 20 YOLOS tenants.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_mq; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
run() {  # tag, podserver_once args...
  tag=$1; shift
  timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d.get('decode_token_latency_ms'), {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/$tag.json $tag
}
M="--mix yolos:20,llama-dec:8 --window 8 --priority-lanes 2"
run cus16_mq8 $M --latency-cus 16 --masked-queues 8 || exit 1
run cus16_mq4 $M --latency-cus 16 --masked-queues 4 || exit 1
run cus32_mq8 $M --latency-cus 32 --masked-queues 8 || exit 1
run cus16_mq6 $M --latency-cus 16 --masked-queues 6 || exit 1
run cus16_mq12 $M --latency-cus 16 --masked-queues 12 || exit 1
