set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r29
mkdir -p $O
for P in 4 8 16 28; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --pods-per-gpu $P --no-control-plane > $O/bench_p$P.log 2>&1 || exit 1
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-control-plane > $O/bench_q8.log 2>&1 && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --pods-per-gpu 16 --no-control-plane > $O/bench_q8_p16.log 2>&1
echo rc=$?
