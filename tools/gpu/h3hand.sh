# h3 plane hand-offs: h3 numerics tests, pod-server GPU tests, default fleet
# (2 rounds) and its kernel profile.  usage (via gpurun): bash tools/gpu/h3hand.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-h3hand}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gemm_h3_gpu.py tests/test_attention_h3_gpu.py tests/test_podserver_gpu.py -x -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "error vs|FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
grep -E "handoff|fc1 -> fc2|passed|failed" $O/tests.log | tail -5
for r in 1 2; do
  timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 > $O/fleet_r$r.json 2> $O/fleet_r$r.err || { echo "fleet failed"; tail -20 $O/fleet_r$r.err; exit 1; }
  timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 --h3-layout 2x2 > $O/fleet22_r$r.json 2> $O/fleet22_r$r.err || { echo "fleet 2x2 failed"; tail -20 $O/fleet22_r$r.err; exit 1; }
  timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 --h3-layout 256x128 > $O/fleet256_r$r.json 2> $O/fleet256_r$r.err || { echo "fleet 256 failed"; tail -20 $O/fleet256_r$r.err; exit 1; }
  echo "r$r 256x128 $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"])' $O/fleet256_r$r.json)"
  echo "r$r 2x2 $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"])' $O/fleet22_r$r.json)"
  echo "r$r $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"], d["server_build_ms_p50"])' $O/fleet_r$r.json)"
done
bash tools/gpu/prof_h3.sh ${1:-h3hand}_prof
