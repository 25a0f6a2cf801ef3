set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/cumask_layouts.py --pods 8 --layouts overlap2,overlap4,shared --out gpurun_out/lay12a.json > gpurun_out/lay12a.log 2>&1 && \
GPU_MAX_HW_QUEUES=1 timeout -k 10 200 python tools/cumask_layouts.py --pods 8 --layouts shared --out gpurun_out/lay12b.json > gpurun_out/lay12b.log 2>&1 && \
GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python tools/cumask_layouts.py --pods 8 --layouts shared --out gpurun_out/lay12c.json > gpurun_out/lay12c.log 2>&1 && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python tools/cumask_layouts.py --pods 8 --layouts shared --out gpurun_out/lay12d.json > gpurun_out/lay12d.log 2>&1 && \
timeout -k 10 300 python tools/cumask_layouts.py --pods 4 --layouts contiguous,overlap2,shared --out gpurun_out/lay12e.json > gpurun_out/lay12e.log 2>&1 && \
timeout -k 10 300 python tools/cumask_layouts.py --pods 16 --layouts overlap2,overlap4,shared --out gpurun_out/lay12f.json > gpurun_out/lay12f.log 2>&1
echo rc=$?
