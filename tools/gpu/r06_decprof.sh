# Decode tenants under rocprofv3 kernel stats: 8 decoders alone, then the
# 20 YOLOS + 8 decoders mix (a segfault there is reported, not retried).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_decprof; mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec8 -o run -- python3 $R/tools/podserver_once.py --mix llama-dec:8 --window 4 > $O/dec8.log 2>&1 || { echo dec8 prof failed; tail -5 $O/dec8.log; exit 1; }
cd $R
python3 - $O/dec8 <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{100*float(r["TotalDurationNs"])/tot:5.1f}% {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:8.1f}us {r["Name"][:90]}')
PY
grep -h '^{' $O/dec8.log | tail -1 | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mix -o run -- python3 $R/tools/podserver_once.py --mix yolos:20,llama-dec:8 --window 4 > $O/mix.log 2>&1 || { echo mix prof failed; tail -5 $O/mix.log; exit 0; }
cd $R
python3 - $O/mix <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{100*float(r["TotalDurationNs"])/tot:5.1f}% {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:8.1f}us {r["Name"][:90]}')
PY
