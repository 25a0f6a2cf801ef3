# Numerics tests of the in-tree kernels, then the 28-tenant fleet A/B of the
# in-tree library ("base") against kernel variants built by
# tools/build_variant.py (build/variants/<name>/libnos_hip.so), 2 rounds.
# usage (via gpurun): bash tools/gpu/ab_variant.sh <tag> <variant> [...]
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gemm_h3_gpu.py tests/test_attention_h3_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then unset NOS_AMD_HIP_LIB; else export NOS_AMD_HIP_LIB=$GRAFT_REPO_ROOT/build/variants/$v/libnos_hip.so; fi
    timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 > $O/fleet_${v}_r$r.json 2> $O/fleet_${v}_r$r.err || { echo "fleet $v failed"; tail -20 $O/fleet_${v}_r$r.err; exit 1; }
    echo "$v r$r $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"])' $O/fleet_${v}_r$r.json)"
  done
done
