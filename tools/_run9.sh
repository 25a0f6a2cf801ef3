set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc1 gpurun_out/pmc2
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/pmc1 -o run --output-format csv -- python tools/kernel_bench.py --only attn,gemm --iters 5 > gpurun_out/pmc1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU --kernel-trace -d gpurun_out/pmc2 -o run --output-format csv -- python tools/kernel_bench.py --only attn,gemm --iters 5 > gpurun_out/pmc2.log 2>&1
echo rc=$?
