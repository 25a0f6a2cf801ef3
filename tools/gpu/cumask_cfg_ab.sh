#!/bin/bash
# Kernel configs for exclusive CU-mask slice pods (persistent grids on): GEMM
# tile policy x fp32 attention tiling, 1 and 7 cumask pods per config.
# usage (GPU box, repo root): bash tools/gpu/cumask_cfg_ab.sh
set -o pipefail
OUT=gpurun_out/cumask_cfg_ab
mkdir -p $OUT
for cfg in "small:w4k32" "latency:w4k32" "throughput:w4k32" "small:w4k64" "small:w4k32o4" "latency:w4k32o4" "latency:w4k64g2"; do
  g=${cfg%%:*}; a=${cfg##*:}
  timeout -k 10 200 python tools/sharing_table.py --modes cumask --pods 1,7 --window 6 \
    --pod-env NOS_AMD_GEMM_F32_POLICY=$g --pod-env NOS_AMD_ATTN_F32_VARIANT=$a \
    --out $OUT/$g-$a.json > $OUT/$g-$a.log 2>&1 || { tail -20 $OUT/$g-$a.log; exit 1; }
done
