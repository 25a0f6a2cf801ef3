#!/bin/bash
# rocprofv3 PMC passes over the fp32 GEMMs (exact-f32 MFMA vs bf16x6 split; tools/gemm_f32_once.py).
# usage (on the GPU box, from the repo root): bash tools/gpu/pmc_gemm_f32.sh
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${PMC_OUT:-pmc_gemm_f32}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CNT in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/pass$i -o run -- python3 $R/tools/gemm_f32_once.py > $OUT/pass$i.log 2>&1 || exit 1
done
