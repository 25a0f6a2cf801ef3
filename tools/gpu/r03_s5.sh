# x6 GEMM timing probe: in-tree kernels vs build/variants/<v> (kernel_bench,
# fp32 x6 GEMMs of YOLOS-small, 128x128 4x1-wave tiles and the policy tile).
# bash tools/gpu/r03_s5.sh <variant>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s5_$1; V=build/variants/$1/libnos_hip.so
mkdir -p $O
for B in 1 8; do for T in 5 -1; do for tag in new var; do
  L=; [ $tag = var ] && L=$V
  NOS_AMD_HIP_LIB=$L timeout -k 10 120 python tools/kernel_bench.py --only gemm --dtype fp32 --f32-math x6 --x6-tile $T \
    --batch $B --iters 20 --rounds 2 --out $O/${tag}_b${B}_t${T}.json > /dev/null 2>> $O/err.log || exit 1
done; done; done
python - $O <<'PY'
import json, sys, glob, os
O = sys.argv[1]
for f in sorted(glob.glob(f"{O}/new_*.json")):
    n = json.load(open(f)); v = json.load(open(f.replace("/new_", "/var_")))
    keys = [k for k in n if k.endswith("_us")]
    print(os.path.basename(f)[4:-5], {k[:-3]: (n[k], v.get(k)) for k in keys})
PY
