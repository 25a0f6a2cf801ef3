# 28-tenant fleet A/B of the pod server's lane count (hardware queues), 2 rounds.
# usage (via gpurun): bash tools/gpu/lanes_ab.sh <tag> <lanes> [...]
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
mkdir -p $O
for r in 1 2; do
  for n in "$@"; do
    timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 --lanes $n > $O/fleet_l${n}_r$r.json 2> $O/fleet_l${n}_r$r.err || { echo "fleet lanes $n failed"; tail -20 $O/fleet_l${n}_r$r.err; exit 1; }
    echo "lanes $n r$r $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"], d["min_done"], d["max_done"])' $O/fleet_l${n}_r$r.json)"
  done
done
