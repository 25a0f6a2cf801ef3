#!/bin/bash
# Round-3 GPU pass: the default 1-GPU bench (headline JSON incl. the latency
# table with persistent-grid CU slices), then the multi-rank launch path folded
# onto the one GPU (2 ranks over gloo, each GPU's slot 0 a DP trainer POD).
# usage (GPU box, repo root): bash tools/gpu/r03_bench.sh [outdir]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_bench}
mkdir -p $O
timeout -k 10 500 python bench.py --json-out $O/bench_n1.json > $O/bench_n1.out 2> $O/bench_n1.err || { tail -30 $O/bench_n1.err; exit 1; }
tail -c 600 $O/bench_n1.out
NOS_AMD_BENCH_FOLD_GPUS=1 NOS_AMD_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 10 --warmup 3 \
  --pods-per-gpu 3 --collective on --table "" --extra-bf16-s 0 --ref-pod-s 0 --json-out $O/bench_n2_fold.json \
  > $O/bench_n2_fold.out 2> $O/bench_n2_fold.err || { tail -30 $O/bench_n2_fold.err; exit 1; }
tail -c 600 $O/bench_n2_fold.out
