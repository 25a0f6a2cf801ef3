# Rehearse bench.py's multi-rank path on a 1-GPU box: 2 and 4 ranks over gloo
# sharing the one GPU (RCCL refuses two ranks on one device), launched exactly
# as the driver launches the 8-GPU run (torch.distributed.run, 127.0.0.1).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-scale_rehearsal}
mkdir -p $O
for N in 2 4; do
  NOS_AMD_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus $N --steps 10 --warmup 3 --pods-per-gpu 2 \
    > $O/bench_n$N.json 2> $O/bench_n$N.err || { tail -20 $O/bench_n$N.err; exit 1; }
  cat $O/bench_n$N.json
done
NOS_AMD_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29610 bench.py --gpus 2 --steps 10 --warmup 3 --pods-per-gpu 2 --collective \
  > $O/bench_n2_coll.json 2> $O/bench_n2_coll.err || { tail -20 $O/bench_n2_coll.err; exit 1; }
cat $O/bench_n2_coll.json
