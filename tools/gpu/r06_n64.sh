# 128 x 64 h3 GEMM tiles (48 KiB: three workgroups per CU, 113 VGPRs) vs the
# 128 x 128 default, both as plain MODE-0 GEMMs (LN hand-off off); layout
# bit-identity test first.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_n64; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_h3_gpu.py -q -k layouts --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head; exit 1; }
tail -1 $O/tests.log
one() {  # tag, args
  local tag=$1; shift
  NOS_AMD_LN_HANDOFF=off timeout -k 10 300 python3 tools/podserver_once.py --tenants 28 --window 10 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['inf_per_s'], d['sclk_mhz'], round(d['inf_per_s']/d['sclk_mhz'],4))" $O/$tag.json $tag
}
for r in 1 2; do
  one x2x2_r$r --h3-layout 2x2 || exit 1
  one n64_r$r --h3-layout 2x2n64 || exit 1
done
