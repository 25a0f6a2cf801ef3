# Round-6 fleets under the current defaults: 28 fp32 YOLOS, 28 bf16 YOLOS, the
# three-family mix (16 YOLOS + 6 ResNet-18 + 6 Llama), and YOLOS + decoders.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_fleets; mkdir -p $O
one() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], {k: v['inf_per_s'] for k, v in (d.get('per_kind') or {}).items()}, d.get('decode_token_latency_ms'), d['sclk_mhz'])" $O/$tag.json $tag
}
one fp32_28 --tenants 28 --window 10 || exit 1
one bf16_28 --tenants 28 --window 10 --dtype bf16 || exit 1
one mix3 --mix yolos:16,resnet:6,llama:6 --window 10 || exit 1
one fp32_28_b --tenants 28 --window 10 || exit 1
one bf16_28_b --tenants 28 --window 10 --dtype bf16 || exit 1
# ring-depth A/B on the MODE-0 GEMMs (LN hand-off off, so every h3 GEMM takes the layout)
for lay in 2x2 2x2k16 4x1r3; do
  NOS_AMD_LN_HANDOFF=off one nolnh_$lay --tenants 28 --window 10 --h3-layout $lay || exit 1
done
