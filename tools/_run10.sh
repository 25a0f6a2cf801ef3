set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/gpu_explore.py --skip masks,probes --out gpurun_out/explore10.json > gpurun_out/explore10.log 2>&1 && \
timeout -k 10 200 python tools/kernel_bench.py --only attn,torch --iters 50 --out gpurun_out/kb10.json > gpurun_out/kb10.log 2>&1 && \
timeout -k 10 300 python tools/tenant_sweep.py --pods 1,4,8,16 --modes cumask,shared --out gpurun_out/sweep10.json > gpurun_out/sweep10.log 2>&1
echo rc=$?
