set -o pipefail
mkdir -p gpurun_out/prof1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --pods-per-gpu 1 --mode exclusive --no-control-plane --steps 10 --warmup 2 > gpurun_out/prof1.log 2>&1 && \
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python tools/tenant_sweep.py --out gpurun_out/sweep_q16.json --steps 20 --pods 4,7,8,16,28 > gpurun_out/sweep_q16.log 2>&1
echo rc=$?
