# Decode kernels with dtype-templated loads (no per-load dtype branch; the first
# GEMV weight chunk and the attention's K / V rows in flight up front): GPU
# tests, then same-box A/B against the committed decode.hip (head), one decoder
# through the generate loop, alternating; 8 decoders.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_decab2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_tenant_programs_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
one() {  # tag, lib ('' = in-tree), args
  t=$1; l=$2; shift 2
  if [ -n "$l" ]; then export NOS_AMD_HIP_LIB=$l; else unset NOS_AMD_HIP_LIB; fi
  timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d.get('decode_token_latency_ms')['mean'], d['sclk_mhz'])" $O/$t.json $t
}
H=$R/build/variants/dec_head/libnos_hip.so
for r in 1 2 3; do
  one cur_r$r "" --mix llama-dec:1 --window 6 --gen-chunk 64 || exit 1
  one head_r$r $H --mix llama-dec:1 --window 6 --gen-chunk 64 || exit 1
done
one cur8 "" --mix llama-dec:8 --window 6 --gen-chunk 16 || exit 1
one head8 $H --mix llama-dec:8 --window 6 --gen-chunk 16 || exit 1
