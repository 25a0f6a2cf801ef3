# h3 attention at 4 waves / SIMD (VGPRs <= 128, two 8-wave workgroups per CU) vs
# 3 (134 VGPRs): attention numerics, then the 28-tenant fleet A/B, alternating.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_attn_occ; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_attention_h3_gpu.py tests/test_gemm_h3_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
one() {  # tag, lib
  NOS_AMD_HIP_LIB=$2 timeout -k 10 300 python3 tools/podserver_once.py --tenants 28 --window 10 > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d['sclk_mhz'])" $O/$1.json $1
}
for r in 1 2; do
  one base_r$r $R/nos_amd/_native/libnos_hip_base.so || exit 1
  one occ4_r$r $R/nos_amd/_native/libnos_hip.so || exit 1
done
bash tools/gpu/r06_decprof.sh
bash tools/gpu/r06_lat3.sh
