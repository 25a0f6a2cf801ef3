# Same-box A/B of the decode kernels' load prefetch, one decoder through the
# generate loop (64 tokens per request), alternating: cur = GEMV + attention
# prefetch, head = neither (the committed decode.hip), attn = attention only.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_decab; mkdir -p $O
one() {  # tag, lib ('' = in-tree)
  if [ -n "$2" ]; then export NOS_AMD_HIP_LIB=$2; else unset NOS_AMD_HIP_LIB; fi
  timeout -k 10 300 python3 tools/podserver_once.py --mix llama-dec:1 --window 6 --gen-chunk 64 > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d.get('decode_token_latency_ms')['mean'], d['sclk_mhz'])" $O/$1.json $1
}
for r in 1 2 3; do
  one cur_r$r "" || exit 1
  one head_r$r $R/build/variants/dec_head/libnos_hip.so || exit 1
  one attn_r$r $R/build/variants/dec_attn/libnos_hip.so || exit 1
done
