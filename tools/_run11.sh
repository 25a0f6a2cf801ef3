set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/cumask_layouts.py --pods 8 > gpurun_out/layouts11.log 2>&1 && \
timeout -k 10 300 python tools/pod_procs.py --pods 8 --modes cumask,shared --iters 40 --out gpurun_out/procs11.json > gpurun_out/procs11.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench11.log 2>&1
echo rc=$?
