# bf16 attention ping-pong schedule: numerics vs lockstep and fp32, kernel time.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s9
mkdir -p $O
timeout -k 10 120 python tools/attn_pp_check.py > $O/check.log 2>&1 || { cat $O/check.log; exit 1; }
cat $O/check.log
for round in 1 2; do for v in lockstep pingpong; do
  timeout -k 10 120 python tools/attn_bench.py --dtype bf16 --bf16-variant $v --batches 1,8 >> $O/attn.jsonl 2>>$O/err.log || exit 1
done; done
cat $O/attn.jsonl
