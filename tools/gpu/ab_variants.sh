# In-tree kernels vs variants (tools/build_variant.py): the h3 attention /
# GEMM numerics tests on the in-tree library, then the 28-tenant fleet of
# every library in rotation, 2 rounds.  usage: bash tools/gpu/ab_variants.sh <tag> <variant>...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q tests/test_attention_h3_gpu.py tests/test_gemm_h3_gpu.py tests/test_ln_handoff_gpu.py --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then unset NOS_AMD_HIP_LIB; else export NOS_AMD_HIP_LIB=$R/build/variants/$v/libnos_hip.so; fi
    timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 > $O/fleet_${v}_r$r.json 2> $O/fleet_${v}_r$r.err || { echo "fleet $v failed"; tail -20 $O/fleet_${v}_r$r.err; exit 1; }
    echo "$v r$r $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"])' $O/fleet_${v}_r$r.json)"
  done
done
unset NOS_AMD_HIP_LIB
bash tools/gpu/pmc_h3.sh $(basename $O)/pmc > /dev/null || exit 1
python3 -c "
import json;d=json.load(open('$O/pmc/summary.json'))
for k,v in d.items():
    if isinstance(v,dict) and 'derived' in v and ('attn' in k or 'gemm_h3' in k): print(k[:50], {a: round(b,2) for a,b in v['derived'].items()})"
