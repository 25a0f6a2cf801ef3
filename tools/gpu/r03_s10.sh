# (1) bench.py's multi-rank path in server mode, 2 ranks folded onto the one
# GPU (gloo between ranks, a pod server + DP trainer pod per rank), launched as
# the driver launches the 8-GPU run; (2) a 2-minute steady-state window of the
# default 28-pod fleet (the reference demo averages over 2 minutes).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s10
mkdir -p $O
NOS_AMD_BENCH_FOLD_GPUS=1 NOS_AMD_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 2 --steps 10 --warmup 3 \
  --pods-per-gpu 6 --extra-bf16-s 0 --ref-pod-s 0 > $O/bench_n2_server_fold.json 2> $O/bench_n2.err \
  || { tail -20 $O/bench_n2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_n2_server_fold.json'));print({k:d[k] for k in ['value','n_gpus','aggregate_inf_per_s','trainer_error']}, d['trainer_pods'] and d['trainer_pods']['rank0'])"
timeout -k 10 600 python bench.py --steps 100 --step-s 1.2 --warmup 10 --table '' --extra-bf16-s 0 \
  --json-out $O/bench_soak.json > /dev/null 2> $O/bench_soak.err || { tail -20 $O/bench_soak.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_soak.json'));print({k:d[k] for k in ['value','aggregate_inf_per_s','window_s','gpu_util_pct','gpu_util_samples','rank0_sclk_mhz','single_pod_inf_per_s']})"
