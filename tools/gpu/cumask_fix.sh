#!/bin/bash
# CU-mask slice isolation with slice-sized persistent grids (round 3):
# 1. numerics: persistent grids are bit-identical to one workgroup per tile;
# 2. the reference demo's latency rows for exclusive CU slices, persistent
#    grids on (default: the pod's budget = its mask's CUs) and off
#    (NOS_AMD_CU_BUDGET=0), plus the unmasked rows for reference.
# usage (GPU box, repo root): bash tools/gpu/cumask_fix.sh [pods] [window_s]
set -o pipefail
PODS=${1:-1,3,5,7,8}
WIN=${2:-6}
OUT=gpurun_out/cumask_fix
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "persistent or fp32" > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 400 python tools/sharing_table.py --modes cumask --pods $PODS --window $WIN \
  --out $OUT/table_persistent.json > $OUT/table_persistent.log 2>&1 || exit 1
timeout -k 10 400 python tools/sharing_table.py --modes cumask --pods $PODS --window $WIN \
  --pod-env NOS_AMD_CU_BUDGET=0 --out $OUT/table_tilegrid.json > $OUT/table_tilegrid.log 2>&1 || exit 1
