set -e
mkdir -p gpurun_out/ab
B="python -u bench.py --table= --ref-pod-s 0 --extra-bf16-s 0"
timeout -k 10 200 $B --json-out gpurun_out/ab/lat1.json > gpurun_out/ab/lat1.log 2>&1
NOS_AMD_GEMM_F32_POLICY=throughput timeout -k 10 200 $B --json-out gpurun_out/ab/thr1.json > gpurun_out/ab/thr1.log 2>&1
timeout -k 10 200 $B --json-out gpurun_out/ab/lat2.json > gpurun_out/ab/lat2.log 2>&1
NOS_AMD_GEMM_F32_POLICY=throughput timeout -k 10 200 $B --json-out gpurun_out/ab/thr2.json > gpurun_out/ab/thr2.log 2>&1
for f in gpurun_out/ab/*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f',d['aggregate_inf_per_s'],d['matrix_pipe_util_pct'],d['value'])"; done
