# Decode kernels with their loads up front (GEMV: the first weight chunk in
# flight while x is staged; decode attention: K and V rows in registers before
# the fresh rows / q staging): GPU tests, decode rates through the generate
# loop, the combine fold again (no host round trip now), and a traced step.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_decprefetch; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_tenant_programs_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
run() {  # tag, podserver_once args...
  tag=$1; shift
  timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d.get('decode_token_latency_ms'), {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/$tag.json $tag
}
run dec1_k64 --mix llama-dec:1 --window 8 --gen-chunk 64 || exit 1
NOS_AMD_FOLD_DECODE_COMBINE=1 run dec1_k64_fold --mix llama-dec:1 --window 8 --gen-chunk 64 || exit 1
run dec1_k64_b --mix llama-dec:1 --window 8 --gen-chunk 64 || exit 1
run dec1_k1 --mix llama-dec:1 --window 8 || exit 1
run dec8_k16 --mix llama-dec:8 --window 8 --gen-chunk 16 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --mix llama-dec:1 --window 3 --gen-chunk 64 > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; rm -rf $O/prof; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 $R/tools/decode_gaps.py $f --tail 5000 > $O/gaps.json && rm -rf $O/prof
head -45 $O/gaps.json
