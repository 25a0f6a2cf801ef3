# LN hand-off round 2: tests, per-shape microbench, fleet A/B of the LN
# hand-off (NOS_AMD_LN_HANDOFF) and the LDS epilogue of plain fp32 GEMMs (--lds-epi)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5_lna2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v tests/test_ln_handoff_gpu.py tests/test_gemm_h3_gpu.py --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/ln_handoff_bench.py > $O/micro.json || exit 1
cat $O/micro.json
for r in 1 2; do
  for cfg in "off:0:off" "on:0:on" "on_lds:1:on"; do
    IFS=: read name epi hand <<< "$cfg"
    NOS_AMD_LN_HANDOFF=$hand timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 --lds-epi $epi > $O/fleet_${name}_r$r.json 2> $O/fleet_${name}_r$r.err || { echo "fleet $name failed"; tail -20 $O/fleet_${name}_r$r.err; exit 1; }
    echo "$name r$r $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"])' $O/fleet_${name}_r$r.json)"
  done
done
