set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r26
mkdir -p $O
timeout -k 10 200 python tools/kernel_bench.py --only attn,gemm --batch 8 --iters 20 --out $O/base_b8.json > $O/base_b8.log 2>&1 && \
NOS_AMD_HIP_LIB=build/variants/asmlds/libnos_hip.so timeout -k 10 100 python tools/kernel_bench.py --only attn --batch 8 --iters 20 --out $O/asmlds_b8.json > $O/asmlds_b8.log 2>&1 && \
NOS_AMD_HIP_LIB=build/variants/pp/libnos_hip.so timeout -k 10 100 python tools/kernel_bench.py --only attn --batch 8 --iters 20 --out $O/pp_b8.json > $O/pp_b8.log 2>&1 && \
timeout -k 10 100 python tools/kernel_bench.py --only attn --batch 1 --iters 50 --out $O/base_b1.json > $O/base_b1.log 2>&1
echo rc=$?
