# fp32 attention tilings: numerics, kernel time at B=1/8, and the 8-pod fleet per tiling
set -e
mkdir -p gpurun_out/attn
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k attention_fp32_exact -x -q --timeout 120 --timeout-method thread > gpurun_out/attn/test.log 2>&1
for v in ${KVARS:-w4k64 w4k64g2 w4k32 w4k32o4 w2k64 w8k64}; do
  timeout -k 10 120 python -u tools/attn_bench.py --dtype fp32 --batches 1,8 --variant $v >> gpurun_out/attn/kernel.jsonl
done
B="python -u bench.py --table= --ref-pod-s 0 --extra-bf16-s 0"
for v in ${FVARS:-w4k64 w4k32 w4k32o4 w2k64 w8k64 w4k64}; do
  NOS_AMD_ATTN_F32_VARIANT=$v timeout -k 10 200 $B --json-out gpurun_out/attn/fleet_$v.json > gpurun_out/attn/fleet_$v.log 2>&1
  python -c "import json;d=json.load(open('gpurun_out/attn/fleet_$v.json'));print('$v',d['aggregate_inf_per_s'],d['matrix_pipe_util_pct'])" | tee -a gpurun_out/attn/fleet.txt
done
cat gpurun_out/attn/kernel.jsonl
