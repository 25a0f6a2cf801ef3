set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r31
mkdir -p $O
timeout -k 10 200 python tools/kernel_bench.py --only gemm --batch 8 --iters 20 --out $O/gemm_b8.json > $O/gemm_b8.log 2>&1
echo rc=$?
