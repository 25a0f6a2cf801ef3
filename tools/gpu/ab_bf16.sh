# bf16 fleet A/B: in-tree kernels vs variants (tools/build_variant.py), the
# bf16 attention / GEMM tests first; 28 bf16 YOLOS tenants, 2 rounds.
# usage (via gpurun): bash tools/gpu/ab_bf16.sh <tag> <variant>...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q tests/test_kernels_gpu.py --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then unset NOS_AMD_HIP_LIB; else export NOS_AMD_HIP_LIB=$R/build/variants/$v/libnos_hip.so; fi
    timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 6 --dtype bf16 > $O/fleet_${v}_r$r.json 2> $O/fleet_${v}_r$r.err || { echo "fleet $v failed"; tail -20 $O/fleet_${v}_r$r.err; exit 1; }
    echo "$v r$r $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"])' $O/fleet_${v}_r$r.json)"
  done
done
