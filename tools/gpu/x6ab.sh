# x6 GEMM: pipelined vs plain K loop -- bit-identity tests, kernel timings at
# the YOLOS shapes (batch 1 and 8), then the pod-server GPU tests and the
# default bench.  usage (via gpurun): bash tools/gpu/x6ab.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-x6ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "x6 or split or qkv or planes" > $O/kernels.log 2>&1 || { echo kernel tests failed; tail -30 $O/kernels.log; exit 1; }
tail -1 $O/kernels.log
for B in 1 8; do
  for P in 1 0; do
    timeout -k 10 200 python tools/kernel_bench.py --pipeline $P --only gemm --dtype fp32 --f32-math x6 --x6-tile 5 --batch $B --iters 20 --rounds 2 --out $O/kb_b${B}_p$P.json > $O/kb_b${B}_p$P.log 2>&1 || { echo kernel_bench failed; tail -20 $O/kb_b${B}_p$P.log; exit 1; }
  done
done
python - $O <<'PY'
import json,sys
O=sys.argv[1]
for B in (1,8):
    a=json.load(open(f"{O}/kb_b{B}_p1.json")); b=json.load(open(f"{O}/kb_b{B}_p0.json"))
    print(B, {k.replace("_us",""): (round(b[k],1), round(a[k],1)) for k in a if k.endswith("_us") and "torch" not in k})
PY
