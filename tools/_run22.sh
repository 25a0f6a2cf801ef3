set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/pytest22.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest22.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/kernel_bench.py --only gemm --iters 50 --out gpurun_out/kb22.json > gpurun_out/kb22.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 > gpurun_out/bench22.log 2>&1
echo rc=$?
