# Fleet A/B of the 28-tenant pod server (tools/podserver_once.py): x6 GEMM
# pipelining, lanes, x6 tile.  usage (via gpurun): bash tools/gpu/fleet_ab.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-fleet_ab}
mkdir -p $O
run() {  # name "args" [ENV=value ...]
  local name=$1 args=$2; shift 2
  env "$@" timeout -k 10 150 python tools/podserver_once.py --tenants 28 --window 6 $args > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -20 $O/$name.err; exit 1; }
  echo "$name $(cat $O/$name.json)"
}
for R in 1 2; do
  run pipe_r$R "--lanes 12 --pipeline 1" X=1 || exit 1
  run plain_r$R "--lanes 12 --pipeline 0" X=1 || exit 1
done
run lanes16 "--lanes 16" X=1 || exit 1
run lanes24 "--lanes 24" X=1 || exit 1
run tile128x64 "--lanes 12" NOS_AMD_X6_TILE=128x64 || exit 1
run tilewide "--lanes 12" NOS_AMD_X6_TILE=wide || exit 1
