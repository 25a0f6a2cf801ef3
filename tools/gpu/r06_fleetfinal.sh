# The last tree's fleets: 28 fp32 YOLOS tenants and 28 bf16 YOLOS tenants on one
# pod server (10 s windows), twice each, alternating.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_fleetfinal; mkdir -p $O
run() {  # tag, podserver_once args...
  tag=$1; shift
  timeout -k 10 300 python3 tools/podserver_once.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d['sclk_mhz'])" $O/$tag.json $tag
}
for r in 1 2; do
  run fp32_r$r --tenants 28 --window 10 || exit 1
  run bf16_r$r --tenants 28 --window 10 --dtype bf16 || exit 1
done
