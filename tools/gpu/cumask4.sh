#!/bin/bash
# BASELINE config 4 on one GPU: 4 CU-mask slices running the bf16 GEMM probe
# (timings) + one rocprofv3 PMC pass split per slice by HSA queue.
# usage (on the GPU box, from the repo root): bash tools/gpu/cumask4.sh
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/cumask4
mkdir -p $OUT
timeout -k 10 200 python tools/cumask_gemm_slices.py run --out $OUT/run.json > $OUT/run.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
  --output-format csv -d $OUT/pmc -o run -- python3 $R/tools/cumask_gemm_slices.py pmc > $OUT/pmc.log 2>&1 || exit 1
cd $R && python tools/cumask_gemm_slices.py summarize $OUT/pmc --out $OUT/summary.json > $OUT/summary.txt 2>&1
