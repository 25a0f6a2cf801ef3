# Graph-correctness diagnostics + x6 kernel timings in one GPU session.
# usage (via gpurun): bash tools/gpu/diag.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-diag}
mkdir -p $O
timeout -k 10 300 python tools/graph_bisect.py > $O/bisect.json 2> $O/bisect.err || { echo bisect failed; tail -20 $O/bisect.err; exit 1; }
cat $O/bisect.json
timeout -k 10 300 python tools/graph_seq.py > $O/seq.json 2> $O/seq.err || { echo seq failed; tail -20 $O/seq.err; exit 1; }
cat $O/seq.json
for B in 1 8; do
  timeout -k 10 200 python tools/kernel_bench.py --only gemm,attn --dtype fp32 --f32-math x6 --x6-tile 5 --batch $B --iters 20 --out $O/kb_x6_b$B.json > $O/kb_b$B.log 2>&1 || { echo kernel_bench failed; tail -20 $O/kb_b$B.log; exit 1; }
  tail -15 $O/kb_b$B.log
done
