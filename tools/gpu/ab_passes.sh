# Fleet A/B over compiler passes (NOS_AMD_SKIP_PASSES): 28 tenants of one
# dtype, the default pass list against each skip set, 2 rounds.
# usage (via gpurun): bash tools/gpu/ab_passes.sh <tag> <fp32|bf16> <skip-set>...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
DT=$2
shift 2
mkdir -p $O
for r in 1 2; do
  for v in none "$@"; do
    NOS_AMD_SKIP_PASSES=$v timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 6 --dtype $DT > $O/fleet_${DT}_${v}_r$r.json 2> $O/fleet_${DT}_${v}_r$r.err || { echo "fleet $v failed"; tail -20 $O/fleet_${DT}_${v}_r$r.err; exit 1; }
    echo "$DT skip=$v r$r $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"])' $O/fleet_${DT}_${v}_r$r.json)"
  done
done
