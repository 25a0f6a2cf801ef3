# the CU-mask contention PMC with 7 co-running masked pods.
# Masked pod 0 (32 CUs, disjoint mask) runs under rocprofv3 --pmc, first alone,
# then while 6 other masked pods (the next 6 disjoint 32-CU masks) infer in the
# background; L2 hit / miss, HBM read / write requests and busy cycles per
# kernel in both cases (TCC counters are device-wide: pod 0's passes see the
# co-tenants' L2 traffic too).  usage (GPU box): bash tools/gpu/cumask_pmc7.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-cumask_pmc7}; mkdir -p $O
mask() { printf "0xffffffff"; for ((z=0; z<$1; z++)); do printf "00000000"; done; }
PASSES=("TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE")
run_passes() {  # $1 = solo | co7
  local i=0
  for CNT in "${PASSES[@]}"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $O/$1_pass$i -o run -- python3 $R/tools/pod_once.py --memory-fraction 0.125 --cu-mask $(mask 0) --iters 40) > $O/$1_pass$i.log 2>&1 || { echo "$1 pass $i failed"; tail -5 $O/$1_pass$i.log; return 1; }
  done
  python3 $R/tools/pmc_summary.py $O --filter "" --out $O/$1_summary.json > /dev/null 2>&1
  python3 - $O $1 <<'PY'
import csv, glob, json, sys
from collections import defaultdict
o, tag = sys.argv[1], sys.argv[2]
agg = defaultdict(lambda: defaultdict(float))
for f in glob.glob(f"{o}/{tag}_pass*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        fam = "gemm_h3" if "gemm_h3" in k else ("attn" if "attn" in k else "other")
        agg[fam][r["Counter_Name"]] += float(r["Counter_Value"])
out = {}
for fam, c in agg.items():
    h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
    out[fam] = {**{k: v for k, v in c.items()}, "l2_hit_pct": round(100 * h / (h + m), 2) if h + m else None}
json.dump(out, open(f"{o}/{tag}_families.json", "w"), indent=1)
print(tag, {f: (v["l2_hit_pct"], int(v.get("TCC_EA0_RDREQ_sum", 0)), int(v.get("GRBM_GUI_ACTIVE", 0))) for f, v in out.items()})
PY
  rm -rf $O/$1_pass1 $O/$1_pass2 $O/$1_pass3
}
run_passes solo || exit 1
pids=()
for k in 1 2 3 4 5 6; do
  timeout -k 5 400 python3 tools/pod_once.py --memory-fraction 0.125 --cu-mask $(mask $k) --seconds 300 > $O/bg$k.log 2>&1 &
  pids+=($!)
done
sleep 45
for k in 1 2 3 4 5 6; do grep -q "kernel config" $O/bg$k.log || { echo "bg pod $k not up"; tail -3 $O/bg$k.log; }; done
run_passes co7; rc=$?
for p in "${pids[@]}"; do kill $p 2>/dev/null; done
wait
exit $rc
