# 120 s sustained window of the default fleet (bench.py, 200 steps of 0.6 s,
# no table / reference pod / bf16 fleet) and BASELINE config 5 composed.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-soak_config5}
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 200 --warmup 5 --table= --ref-pod-s 0 --extra-bf16-s 0 --json-out $O/soak.json > $O/soak.log 2>&1 || { echo soak failed; tail -20 $O/soak.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/soak.json'));print({k:d.get(k) for k in ('aggregate_inf_per_s','window_s','gpu_util_pct','rank0_sclk_mhz','matrix_pipe_util_pct')})"
timeout -k 10 900 python bench.py --quota --composed --json-out $O/composed.json > $O/composed.log 2>&1 || { echo composed failed; tail -30 $O/composed.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/composed.json'));print({k:(d[k].get('trainer') if isinstance(d[k],dict) else d[k]) for k in d if k.startswith('phase')})"
