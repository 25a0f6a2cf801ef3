# 8-pod fp32 fleet A/B over environment settings the pods inherit:
#   CONFIGS="name:VAR=val,VAR=val name2:..." bash tools/gpu/ab_fleet_env.sh
# (an empty setting list = the defaults).  Each run: bench.py without the
# latency table, reference pod or bf16 fleet; results in gpurun_out/fleet_ab/.
set -e
mkdir -p gpurun_out/fleet_ab
for cfg in $CONFIGS; do
  name=${cfg%%:*}; sets=${cfg#*:}
  envs=$(echo "$sets" | tr ',' ' ')
  env $envs timeout -k 10 200 python -u bench.py --table= --ref-pod-s 0 --extra-bf16-s 0 \
      --json-out gpurun_out/fleet_ab/$name.json > gpurun_out/fleet_ab/$name.log 2>&1
  python -c "import json;d=json.load(open('gpurun_out/fleet_ab/$name.json'));print('$name','$sets',d['aggregate_inf_per_s'],d['matrix_pipe_util_pct'])" | tee -a gpurun_out/fleet_ab/results.txt
done
