# Why decode on CU-reserved latency lanes is slow: one decoder alone with 0 / 16
# / 64 reserved CUs (priority lanes), and one decoder alone on a CU-masked
# normal lane set.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_lat2; mkdir -p $O
for cfg in "2 0" "2 16" "2 64"; do
  set -- $cfg
  tag=pl$1_cu$2
  timeout -k 10 200 python3 tools/podserver_once.py --mix llama-dec:1 --window 4 --priority-lanes $1 --latency-cus $2 > $O/dec1_$tag.json 2> $O/dec1_$tag.err || { echo "dec1 $tag failed"; tail -5 $O/dec1_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('dec1', sys.argv[2], d['inf_per_s'], d['decode_token_latency_ms'], d['sclk_mhz'])" $O/dec1_$tag.json $tag
done
# CU-mask contention mitigation A/B: the bench's cumask rows (1 and 7 masked
# 32-CU pods, one GPU process each) under GEMM configurations that shrink a
# slice's L2 working set or hide more miss latency.
set -o pipefail
export TMPDIR=/tmp
O=$R/gpurun_out/r06_cumask_ab; mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 420 python -u bench.py --steps 3 --warmup 1 --table 1,7 --table-modes cumask --extra-bf16-s 0 --ref-pod-s 0 --json-out $O/$tag.json > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -8 $O/$tag.log; return 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],[(r['pods'],r['inf_per_s'],r.get('latency_vs_solo_at_solo_clock'),r.get('sclk_mhz')) for r in d['latency_table']])" $O/$tag.json $tag
}
run default NOS_AMD_H3_LAYOUT=2x2 || exit 1
run r3_nolnh NOS_AMD_H3_LAYOUT=4x1r3 NOS_AMD_LN_HANDOFF=off || exit 1
run t256_nolnh NOS_AMD_H3_LAYOUT=256x128 NOS_AMD_LN_HANDOFF=off || exit 1
run nolnh NOS_AMD_LN_HANDOFF=off || exit 1
