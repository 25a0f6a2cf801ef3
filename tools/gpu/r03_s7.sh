# Pod-server fleet A/B of kernel configs and lane counts with the current
# kernels (tools/podserver_once.py: 28 tenants in one process, 8 s window).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s7
mkdir -p $O
for round in 1 2; do
  for cfg in default NOS_AMD_X6_TILE=wide NOS_AMD_X6_TILE=256x128 NOS_AMD_X6_TILE=128x64 NOS_AMD_ATTN_F32_VARIANT=x6 lanes=16 lanes=8; do
    lanes=12; envs=()
    case $cfg in lanes=*) lanes=${cfg#lanes=};; default) ;; *) envs=("$cfg");; esac
    env "${envs[@]}" timeout -k 10 120 python tools/podserver_once.py --tenants 28 --lanes $lanes --window 8 \
      2>>$O/err.log | sed "s/^{/{\"cfg\": \"$cfg\", \"round\": $round, /" >> $O/fleet_ab.jsonl || exit 1
  done
done
python - $O/fleet_ab.jsonl <<'PY'
import json, sys, collections
r = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    d = json.loads(ln); r[d["cfg"]].append(d["inf_per_s"])
for k, v in r.items(): print(k, v)
PY
