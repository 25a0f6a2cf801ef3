# Reserved latency CUs with more hardware queues than streams (queue sharing test).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_lat3; mkdir -p $O
for cfg in "16 18" "16 32" "0 32"; do
  set -- $cfg
  tag=cu$1_q$2
  timeout -k 10 300 python3 tools/podserver_once.py --mix yolos:20,llama-dec:8 --window 8 --priority-lanes 2 --latency-cus $1 --hw-queues $2 > $O/mix_$tag.json 2> $O/mix_$tag.err || { echo "mix $tag failed"; tail -5 $O/mix_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('mix', sys.argv[2], d['inf_per_s'], d['decode_token_latency_ms'], {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/mix_$tag.json $tag
done
