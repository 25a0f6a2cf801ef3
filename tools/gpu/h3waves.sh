# h3 attention 4- vs 8-wave workgroups: bit-identity test, then the fleet A/B.
# usage (via gpurun): bash tools/gpu/h3waves.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-h3waves}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attention_h3_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for w in 4 8; do
    timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 --h3-attn-waves $w > $O/fleet_w${w}_r$r.json 2> $O/fleet_w${w}_r$r.err || { echo "fleet $w failed"; tail -20 $O/fleet_w${w}_r$r.err; exit 1; }
    echo "waves $w r$r $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"])' $O/fleet_w${w}_r$r.json)"
  done
done
