# h3 plane hand-offs: h3 numerics tests, pod-server GPU tests, the 28-tenant
# fleet under every h3 GEMM layout (2 rounds) and the default's kernel profile.
# usage (via gpurun): bash tools/gpu/h3hand.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-h3hand}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gemm_h3_gpu.py tests/test_attention_h3_gpu.py tests/test_podserver_gpu.py -x -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "error vs|FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
grep -E "fc1 -> fc2|passed|failed" $O/tests.log | tail -3
for r in 1 2; do
  for lay in 4x1 2x2 256x128 4x1r3 4x1k16 2x2k16; do
    timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 --h3-layout $lay > $O/fleet_${lay}_r$r.json 2> $O/fleet_${lay}_r$r.err || { echo "fleet $lay failed"; tail -20 $O/fleet_${lay}_r$r.err; exit 1; }
    echo "r$r $lay $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"], d["server_build_ms_p50"])' $O/fleet_${lay}_r$r.json)"
  done
done
bash tools/gpu/prof_h3.sh ${1:-h3hand}_prof
