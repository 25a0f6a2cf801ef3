#!/bin/bash
# rocprofv3 PMC passes over the bf16 GEMM configs and hipBLASLt (tools/gemm_once.py).
# usage (on the GPU box, from the repo root): bash tools/gpu/pmc_gemm.sh
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${PMC_OUT:-pmc_gemm}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CNT in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $OUT/pass$i -o run -- python3 $R/tools/gemm_once.py > $OUT/pass$i.log 2>&1 || exit 1
done
