# CU-mask contention mitigation A/B: the bench's cumask rows (1 and 7 masked
# 32-CU pods, one GPU process each) under GEMM configurations that shrink a
# slice's L2 working set or hide more miss latency.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_cumask_ab; mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 420 python -u bench.py --steps 3 --warmup 1 --table 1,7 --table-modes cumask --extra-bf16-s 0 --ref-pod-s 0 --json-out $O/$tag.json > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -8 $O/$tag.log; return 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],[(r['pods'],r['inf_per_s'],r.get('latency_vs_solo_at_solo_clock'),r.get('sclk_mhz')) for r in d['latency_table']])" $O/$tag.json $tag
}
run default NOS_AMD_H3_LAYOUT=2x2 || exit 1
run r3_nolnh NOS_AMD_H3_LAYOUT=4x1r3 NOS_AMD_LN_HANDOFF=off || exit 1
run t256_nolnh NOS_AMD_H3_LAYOUT=256x128 NOS_AMD_LN_HANDOFF=off || exit 1
run nolnh NOS_AMD_LN_HANDOFF=off || exit 1
