set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest15.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest15.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/kernel_bench.py --only attn,gemm --iters 50 --out gpurun_out/kb15.json > gpurun_out/kb15.log 2>&1
echo rc=$?
