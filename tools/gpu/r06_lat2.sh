# Why decode on CU-reserved latency lanes is slow: one decoder alone with 0 / 16
# / 64 reserved CUs (priority lanes), and one decoder alone on a CU-masked
# normal lane set.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_lat2; mkdir -p $O
for cfg in "2 0" "2 16" "2 64"; do
  set -- $cfg
  tag=pl$1_cu$2
  timeout -k 10 200 python3 tools/podserver_once.py --mix llama-dec:1 --window 4 --priority-lanes $1 --latency-cus $2 > $O/dec1_$tag.json 2> $O/dec1_$tag.err || { echo "dec1 $tag failed"; tail -5 $O/dec1_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('dec1', sys.argv[2], d['inf_per_s'], d['decode_token_latency_ms'], d['sclk_mhz'])" $O/dec1_$tag.json $tag
done
