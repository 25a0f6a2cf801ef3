# The decode split combine folded into the decode attention launch (last
# workgroup per K / V head, device-scope counters): GPU tests, decode rates
# with / without the fold (NOS_AMD_SKIP_PASSES=decode_combine), the YOLOS mix;
# then reserved-CU latency lanes with lo_only throughput lanes (r06_mq2.sh).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_dsync; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_tenant_programs_gpu.py tests/test_decode_tenants.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
run() {  # tag, podserver_once args...
  tag=$1; shift
  timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d.get('decode_token_latency_ms'), {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/$tag.json $tag
}
run dec1 --mix llama-dec:1 --window 8 || exit 1
NOS_AMD_SKIP_PASSES=decode_combine run dec1_nofold --mix llama-dec:1 --window 8 || exit 1
run dec1_b --mix llama-dec:1 --window 8 || exit 1
run dec8 --mix llama-dec:8 --window 8 || exit 1
NOS_AMD_SKIP_PASSES=decode_combine run dec8_nofold --mix llama-dec:8 --window 8 || exit 1
run mix --mix yolos:20,llama-dec:8 --window 8 || exit 1
M="--mix yolos:20,llama-dec:8 --window 8"
run pl4_cus16 $M --priority-lanes 4 --latency-cus 16 --masked-queues 8 || exit 1
run pl2_cus16 $M --priority-lanes 2 --latency-cus 16 --masked-queues 8 || exit 1
run pl4_cus32 $M --priority-lanes 4 --latency-cus 32 --masked-queues 8 || exit 1
run pl8_cus32 $M --priority-lanes 8 --latency-cus 32 --masked-queues 6 || exit 1
