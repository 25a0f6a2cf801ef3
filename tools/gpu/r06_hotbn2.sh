# Residual GEMMs on 128 x 64 tiles (LN-GEMMs 128 x 128) vs all 128 x 128.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_hotbn2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ln_handoff_gpu.py tests/test_gemm_h3_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
one() {  # tag, bn
  NOS_AMD_H3_HOT_BN=$2 timeout -k 10 300 python3 tools/podserver_once.py --tenants 28 --window 10 > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d['sclk_mhz'], round(d['inf_per_s']/d['sclk_mhz'],4))" $O/$1.json $1
}
for r in 1 2; do
  one bn128_r$r 128 || exit 1
  one bn64_r$r 64 || exit 1
done
