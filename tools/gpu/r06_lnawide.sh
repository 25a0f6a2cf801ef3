# fc1-class LN-GEMMs on 128 x 256 tiles with 8 waves vs 128 x 128: bit-identity
# test, then the 28-tenant fleet A/B, alternating.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_lnawide; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ln_handoff_gpu.py tests/test_gemm_h3_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
one() {  # tag, on|off
  timeout -k 10 300 python3 tools/podserver_once.py --tenants 28 --window 10 --h3-lna-wide $2 > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d['sclk_mhz'], round(d['inf_per_s']/d['sclk_mhz'],4))" $O/$1.json $1
}
for r in 1 2; do
  one off_r$r off || exit 1
  one on_r$r on || exit 1
done
