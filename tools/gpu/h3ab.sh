# fp16x3 attention + GEMM: numerics tests, x6 plane regressions, GEMM kernel
# times and the 28-tenant fleet A/B against the x6 kernels.
# usage (via gpurun): bash tools/gpu/h3ab.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-h3ab}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_attention_h3_gpu.py tests/test_gemm_h3_gpu.py -x -v -s --timeout 200 --timeout-method thread > $O/h3_tests.log 2>&1 || { echo h3 tests failed; grep -E "error vs|FAIL|Error|assert" $O/h3_tests.log | head -30; tail -30 $O/h3_tests.log; exit 1; }
grep -E "error vs fp64|error vs|passed|failed" $O/h3_tests.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "planes or qkv or attention_fp32" > $O/kernels.log 2>&1 || { echo kernel tests failed; tail -30 $O/kernels.log; exit 1; }
tail -1 $O/kernels.log
for m in x6 h3; do
  timeout -k 10 200 python tools/kernel_bench.py --only gemm --dtype fp32 --f32-math $m --x6-tile 5 --batch 1 --iters 20 --rounds 2 --out $O/kb_$m.json > $O/kb_$m.log 2>&1 || { echo "kernel_bench $m failed"; tail -20 $O/kb_$m.log; exit 1; }
done
python - $O <<'PY'
import json,sys
O=sys.argv[1]
for m in ("x6","h3"):
    a=json.load(open(f"{O}/kb_{m}.json"))
    print(m, {k.replace("_us",""): round(a[k],1) for k in a if k.endswith("_us") and "torch" not in k})
PY
for r in 1 2; do
  for cfg in x6:x6n x6:h3n h3:h3n; do
    m=${cfg%%:*}; v=${cfg##*:}
    NOS_AMD_F32_MATH=$m NOS_AMD_ATTN_F32_VARIANT=$v timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 > $O/fleet_${m}_${v}_r$r.json 2> $O/fleet_${m}_${v}_r$r.err || { echo "fleet $cfg failed"; tail -20 $O/fleet_${m}_${v}_r$r.err; exit 1; }
    echo "$cfg r$r $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["inf_per_s"], d["sclk_mhz"])' $O/fleet_${m}_${v}_r$r.json)"
  done
done
