#!/bin/bash
# Whole-GPU reference pod A/B over environment settings the pod inherits:
#   CONFIGS="name:VAR=val,VAR=val name2:..." bash tools/gpu/ab_refpod_env.sh
# Each run: bench.py with a 10 s reference-pod window and a short 8-pod window;
# results (single_pod_inf_per_s) in gpurun_out/refpod_ab/.
set -e
mkdir -p gpurun_out/refpod_ab
for cfg in $CONFIGS; do
  name=${cfg%%:*}; sets=${cfg#*:}
  envs=$(echo "$sets" | tr ',' ' ')
  env $envs timeout -k 10 200 python -u bench.py --table= --ref-pod-s 10 --extra-bf16-s 0 --steps 3 --warmup 1 \
      --json-out gpurun_out/refpod_ab/$name.json > gpurun_out/refpod_ab/$name.log 2>&1
  python -c "import json;d=json.load(open('gpurun_out/refpod_ab/$name.json'));print('$name','$sets',d['single_pod_inf_per_s'],d['aggregate_inf_per_s'])" | tee -a gpurun_out/refpod_ab/results.txt
done
