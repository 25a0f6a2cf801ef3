set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof16
timeout -k 10 300 python tools/slice_probe.py --out gpurun_out/slice_probe16.json > gpurun_out/slice16.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof16 -o bench --output-format csv -- python bench.py --steps 10 --warmup 2 > gpurun_out/prof16.log 2>&1
echo rc=$?
