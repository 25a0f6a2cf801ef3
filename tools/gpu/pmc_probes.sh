#!/bin/bash
# rocprofv3 PMC passes over the gpuagent probe kernels (one counter group per run).
# usage (on the GPU box, from the repo root): bash tools/gpu/pmc_probes.sh [script.py args...]
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/pmc_probes
SCRIPT=${1:-tools/probe_kernels_once.py}
shift || true
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CNT in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum" "SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $OUT/pass$i -o run -- python3 $R/$SCRIPT "$@" > $OUT/pass$i.log 2>&1 || exit 1
done
