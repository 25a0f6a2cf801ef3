# rocprofv3 PMC passes over the 28-tenant YOLOS fp32 pod-server fleet itself
# (tools/podserver_once.py: server + clients in one process, so the counters
# are the fleet's own kernel instantiations and shapes; dispatches serialise
# under --pmc).  usage (GPU box, repo root): bash tools/gpu/pmc_fleet.sh <tag> [tenants]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pmc_fleet}; N=${2:-28}; mkdir -p $O
cd /tmp
i=0
for CNT in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $O/pass$i -o run -- python3 $R/tools/podserver_once.py --tenants $N --window 3 --warmup 2 > $O/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
done
cd $R
python3 tools/pmc_summary.py $O --out $O/summary.json > /dev/null && rm -rf $O/pass1 $O/pass2 && python3 - $O/summary.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
rows=sorted(d.items(), key=lambda kv: -kv[1]["counters"].get("SQ_BUSY_CYCLES",0))
for k,v in rows[:8]: print(k[:100], {a: round(b,2) for a,b in v["derived"].items()})
PY
