set -o pipefail
export TMPDIR=/tmp
V=build/variants/ring3/libnos_hip.so
timeout -k 10 200 python tools/kernel_bench.py --only gemm --iters 50 --out gpurun_out/kb21_base.json > gpurun_out/kb21.log 2>&1 && \
NOS_AMD_HIP_LIB=$V timeout -k 10 200 python tools/kernel_bench.py --only gemm --iters 50 --out gpurun_out/kb21_ring3.json >> gpurun_out/kb21.log 2>&1 && \
NOS_AMD_HIP_LIB=$V timeout -k 10 300 python tests/../bench.py --steps 20 > gpurun_out/bench21_ring3.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 > gpurun_out/bench21_base.log 2>&1
echo rc=$?
