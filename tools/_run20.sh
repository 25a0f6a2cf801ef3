set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/gemm_sweep.py --out gpurun_out/gemm_sweep20.json > gpurun_out/gemm_sweep20.log 2>&1 && \
timeout -k 10 300 python tools/kernel_bench.py --iters 50 --out gpurun_out/kb20.json > gpurun_out/kb20.log 2>&1
echo rc=$?
