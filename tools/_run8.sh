set -o pipefail
timeout -k 10 200 python tools/kernel_bench.py --iters 50 > gpurun_out/kb8.log 2>&1 && \
timeout -k 10 300 python tools/tenant_sweep.py --out gpurun_out/sweep8.json --steps 20 --pods 1,4,8,16 > gpurun_out/sweep8.log 2>&1
echo rc=$?
