#!/bin/bash
# rocprofv3 PMC passes (wait / issue breakdown) over one fp32 and one bf16 attention call.
# usage (on the GPU box, from the repo root): bash tools/gpu/pmc_attn.sh [B] [fp32 variant] [dtypes]
set -o pipefail
R=$PWD
B=${1:-8}
V=${2:-auto}
DT=${3:-fp32,bf16}
OUT=$R/gpurun_out/pmc_attn_${V}_b$B
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CNT in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $OUT/pass$i -o run -- python3 $R/tools/attn_once.py --B $B --variant $V --dtypes $DT > $OUT/pass$i.log 2>&1 || exit 1
done
