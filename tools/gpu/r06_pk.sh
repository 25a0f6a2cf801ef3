# Packed-fp32 GEMM epilogues (+ the residual GEMMs' 3-deep ring option):
# numerics tests, then the 28-tenant fp32 fleet A/B against the previous
# library (libnos_hip_base.so), alternating.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_pk; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_h3_gpu.py tests/test_ln_handoff_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
NOS_AMD_H3_HOT_RING=3 timeout -k 10 600 python -u -m pytest tests/test_ln_handoff_gpu.py -q --timeout 300 --timeout-method thread > $O/tests_r3.log 2>&1 || { echo r3 tests failed; grep -E "Error|assert|FAILED|failed" $O/tests_r3.log | head -30; exit 1; }
tail -1 $O/tests_r3.log
one() {  # tag, lib, extra args
  local tag=$1 lib=$2; shift 2
  NOS_AMD_HIP_LIB=$lib timeout -k 10 300 python3 tools/podserver_once.py --tenants 28 --window 10 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d['sclk_mhz'])" $O/$tag.json $tag
}
for r in 1 2; do
  one base_r$r $R/nos_amd/_native/libnos_hip_base.so || exit 1
  one pk_r$r $R/nos_amd/_native/libnos_hip.so || exit 1
  one pk_ring3_r$r $R/nos_amd/_native/libnos_hip.so --h3-hot-ring 3 || exit 1
done
