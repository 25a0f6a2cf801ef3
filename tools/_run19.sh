set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/gemm_sweep.py --out gpurun_out/gemm_sweep19.json > gpurun_out/gemm_sweep19.log 2>&1
echo rc=$?
