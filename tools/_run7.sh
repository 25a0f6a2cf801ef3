set -o pipefail
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python bench.py --pods-per-gpu 1 --mode exclusive --no-control-plane --steps 10 --warmup 2 > gpurun_out/prof2.log 2>&1 && \
timeout -k 10 300 python tools/tenant_sweep.py --out gpurun_out/sweep3.json --steps 20 --pods 1,4,8,16 > gpurun_out/sweep3.log 2>&1
echo rc=$?
