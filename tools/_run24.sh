set -o pipefail
export TMPDIR=/tmp
V=build/variants/asmlds/libnos_hip.so
NOS_AMD_HIP_LIB=$V timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "attention or yolos" > gpurun_out/pytest24.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest24.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/kernel_bench.py --only attn --iters 100 --out gpurun_out/kb24_base.json > gpurun_out/kb24_base.log 2>&1 && \
NOS_AMD_HIP_LIB=$V timeout -k 10 200 python tools/kernel_bench.py --only attn --iters 100 --out gpurun_out/kb24_var.json > gpurun_out/kb24_var.log 2>&1 && \
NOS_AMD_HIP_LIB=$V timeout -k 10 300 python bench.py --steps 20 > gpurun_out/bench24_var.log 2>&1
echo rc=$?
