# Decode GEMV grid cap 16 workgroups per CU (was 4): the vocabulary head runs its 4000
# column groups at once; GPU tests, same-box A/B against the previous decode.hip (015).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_cap; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
one() {  # tag, lib ('' = in-tree), args
  t=$1; l=$2; shift 2
  if [ -n "$l" ]; then export NOS_AMD_HIP_LIB=$l; else unset NOS_AMD_HIP_LIB; fi
  timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d.get('decode_token_latency_ms')['mean'], d['sclk_mhz'])" $O/$t.json $t
}
H=$R/build/variants/dec_015/libnos_hip.so
for r in 1 2 3; do
  one new_r$r "" --mix llama-dec:1 --window 6 --gen-chunk 64 || exit 1
  one old_r$r $H --mix llama-dec:1 --window 6 --gen-chunk 64 || exit 1
done
one new8 "" --mix llama-dec:8 --window 6 --gen-chunk 16 || exit 1
one old8 $H --mix llama-dec:8 --window 6 --gen-chunk 16 || exit 1
