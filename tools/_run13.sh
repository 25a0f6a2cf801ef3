set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest13.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest13.log
timeout -k 10 200 python tools/kernel_bench.py --only attn --iters 50 --out gpurun_out/kb13.json > gpurun_out/kb13.log 2>&1 && \
timeout -k 10 300 python tools/cumask_layouts.py --pods 8 --layouts contiguous,shared --out gpurun_out/lay13.json > gpurun_out/lay13.log 2>&1
echo rc=$?
