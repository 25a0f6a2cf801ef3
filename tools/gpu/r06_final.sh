# Round-6 final check: the driver's round-end steps (pytest -m gpu, smoke(),
# default bench.py), fleet kernel stats, and the 20 YOLOS + 8 decoders mix
# under kernel stats (the summary CSV only; traces deleted).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r06_final}; mkdir -p $O
bash tools/gpu/full_check.sh ${1:-r06_final} || exit 1
cd /tmp
# graph packet capture off for this trace only: with it the traced mix segfaults in hipGraphLaunch (r06_mixdiag)
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mixprof -o run -- python3 $R/tools/podserver_once.py --mix yolos:20,llama-dec:8 --window 4 > $O/mixprof.log 2>&1 || { echo mix prof failed; tail -5 $O/mixprof.log; exit 0; }
cd $R
f=$(find $O/mixprof -name "*kernel_stats.csv" | head -1); cp $f $O/mix_kernel_stats.csv; rm -rf $O/mixprof
grep -h '^{' $O/mixprof.log | tail -1 | cut -c1-400
python3 - $O/mix_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(f'{100*float(r["TotalDurationNs"])/tot:5.1f}% {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:8.1f}us {r["Name"][:90]}')
PY
