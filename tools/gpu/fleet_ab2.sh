# Fleet A/B of x6 GEMM wave layouts with the pipelined K loop (power-bound
# fleet: fewer LDS reads per MFMA may buy clock).  usage: bash tools/gpu/fleet_ab2.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-fleet_ab2}
mkdir -p $O
run() {  # name "args" [ENV=value ...]
  local name=$1 args=$2; shift 2
  env "$@" timeout -k 10 150 python tools/podserver_once.py --tenants 28 --window 6 $args > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -20 $O/$name.err; exit 1; }
  echo "$name $(cat $O/$name.json)"
}
for R in 1 2; do
  run default_r$R "--lanes 12" X=1 || exit 1
  run t128x128_2x2_r$R "--lanes 12" NOS_AMD_X6_TILE=0 || exit 1
  run t256x128_8x1_r$R "--lanes 12" NOS_AMD_X6_TILE=7 || exit 1
done
