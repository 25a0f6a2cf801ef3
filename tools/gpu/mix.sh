# Heterogeneous tenants on one pod server: YOLOS-small fp32 + BERT-base-shaped
# fp32 encoder + bf16 GEMM-MLP probe, vs the same server with YOLOS only.
# usage (via gpurun): bash tools/gpu/mix.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-mix}
mkdir -p $O
for spec in yolos:28 yolos:20,bert:4,mlp:4 bert:8; do
  echo "== $spec"
  timeout -k 10 240 python -u tools/podserver_once.py --mix $spec --window 8 > $O/mix_${spec//[:,]/_}.json 2> $O/mix_${spec//[:,]/_}.err || { echo "mix $spec failed"; tail -30 $O/mix_${spec//[:,]/_}.err; exit 1; }
  cat $O/mix_${spec//[:,]/_}.json
done
