# The decode combine folded into the O-projection GEMV (sdpa_cache partials +
# gemv_partials, default): GPU tests, then same-box A/B against the combine
# launch (NOS_AMD_SKIP_PASSES=combine_gemv), one decoder through the generate
# loop, alternating; 8 decoders; the mix.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_partials; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_tenant_programs_gpu.py tests/test_program_fuzz_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
one() {  # tag, skip passes, args
  t=$1; k=$2; shift 2
  NOS_AMD_SKIP_PASSES=$k timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d.get('decode_token_latency_ms')['mean'], {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/$t.json $t
}
for r in 1 2 3; do
  one fold_r$r "" --mix llama-dec:1 --window 6 --gen-chunk 64 || exit 1
  one launch_r$r combine_gemv --mix llama-dec:1 --window 6 --gen-chunk 64 || exit 1
done
one fold8 "" --mix llama-dec:8 --window 6 --gen-chunk 16 || exit 1
one launch8 combine_gemv --mix llama-dec:8 --window 6 --gen-chunk 16 || exit 1
one fold_k1 "" --mix llama-dec:1 --window 6 || exit 1
one mix "" --mix yolos:20,llama-dec:8 --window 8 || exit 1
