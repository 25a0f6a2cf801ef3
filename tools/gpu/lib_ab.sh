# A/B of the in-tree kernels against a variant library (tools/build_variant.py):
# bash tools/gpu/lib_ab.sh <tag> <variant-name> [what: gemm|attn]
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; V=build/variants/$2/libnos_hip.so; W=${3:-gemm}
mkdir -p $O
NOS_AMD_HIP_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_var.log 2>&1
rc=$?; tail -2 $O/pytest_var.log; [ $rc -eq 0 ] || exit $rc
for R in 1 2; do for B in 1 8; do
  NOS_AMD_HIP_LIB=$V timeout -k 10 120 python tools/kernel_bench.py --only $W --batch $B --iters 20 --rounds 2 --out $O/var_b${B}_r$R.json > /dev/null 2>> $O/err.log || exit 1
  timeout -k 10 120 python tools/kernel_bench.py --only $W --batch $B --iters 20 --rounds 2 --out $O/new_b${B}_r$R.json > /dev/null 2>> $O/err.log || exit 1
done; done
for R in 1 2; do
  NOS_AMD_HIP_LIB=$V timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/bench_var_r$R.json 2>>$O/err.log || exit 1
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/bench_new_r$R.json 2>>$O/err.log || exit 1
done
python - $O <<'PY'
import json,sys,glob
O=sys.argv[1]
for B in (1,8):
    for tag in ("var","new"):
        ds=[json.load(open(f)) for f in sorted(glob.glob(f"{O}/{tag}_b{B}_r*.json"))]
        keys=[k for k in ds[0] if k.endswith("_us") and "torch" not in k and "sdpa" not in k]
        print(B, tag, {k[:-3]: round(min(d[k] for d in ds),1) for k in keys})
for tag in ("var","new"):
    print(tag, [json.load(open(f))["value"] for f in sorted(glob.glob(f"{O}/bench_{tag}_r*.json"))])
PY

