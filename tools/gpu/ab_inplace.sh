# In-tree kernels vs a variant (tools/build_variant.py): h3 numerics tests,
# tools/ln_handoff_bench.py timings for both, 28-tenant fleet x2 rounds.
# usage (via gpurun): bash tools/gpu/ab_inplace.sh <tag> <variant>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
V=$2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q tests/test_ln_handoff_gpu.py tests/test_gemm_h3_gpu.py tests/test_tenant_programs_gpu.py tests/test_tenant_ops_gpu.py tests/test_podserver_gpu.py --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/ln_handoff_bench.py > $O/micro.json || exit 1
cat $O/micro.json
NOS_AMD_HIP_LIB=$R/build/variants/$V/libnos_hip.so timeout -k 10 200 python tools/ln_handoff_bench.py > $O/micro_$V.json || exit 1
cat $O/micro_$V.json
for r in 1 2; do
  for v in base $V; do
    if [ "$v" = base ]; then unset NOS_AMD_HIP_LIB; else export NOS_AMD_HIP_LIB=$R/build/variants/$v/libnos_hip.so; fi
    timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 > $O/fleet_${v}_r$r.json 2> $O/fleet_${v}_r$r.err || { echo "fleet $v failed"; tail -20 $O/fleet_${v}_r$r.err; exit 1; }
    echo "$v r$r $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"])' $O/fleet_${v}_r$r.json)"
  done
done
