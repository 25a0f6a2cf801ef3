# Fleet A/B over one environment variable the server process reads at start:
# 28 tenants of one dtype, 2 rounds per value.
# usage (via gpurun): bash tools/gpu/ab_env.sh <tag> <fp32|bf16> <VAR> <value>...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
DT=$2
VAR=$3
shift 3
mkdir -p $O
for r in 1 2; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 6 --dtype $DT > $O/fleet_${DT}_${v}_r$r.json 2> $O/fleet_${DT}_${v}_r$r.err || { echo "fleet $v failed"; tail -20 $O/fleet_${DT}_${v}_r$r.err; exit 1; }
    echo "$DT $VAR=$v r$r $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"])' $O/fleet_${DT}_${v}_r$r.json)"
  done
done
