# Wide plane stores (EPI_WIDE) A/B: h3 numerics tests, per-shape timings with
# and without, the 28-tenant fleet A/B, then the decode-tenant measurements.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_wide; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q tests/test_gemm_h3_gpu.py tests/test_ln_handoff_gpu.py tests/test_podserver_gpu.py --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 0 1; do
  NOS_AMD_H3_WIDE_PLANES=$v timeout -k 10 300 python3 tools/ln_handoff_bench.py > $O/lnb_$v.json 2> $O/lnb_$v.err || { echo lnb failed; tail -5 $O/lnb_$v.err; exit 1; }
  echo "wide=$v $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print({b: {k: v for k, v in d[b].items() if k in ('qkv','fc1')} for b in d})" $O/lnb_$v.json)"
done
bash tools/gpu/ab_env.sh r06_wide/ab fp32 NOS_AMD_H3_WIDE_PLANES 0 1 || exit 1
bash tools/gpu/decode_fleet.sh r06_dec_fleet
