# r06_mixdiag: the 20 YOLOS + 8 decoders mix runs without the profiler and
# 8 decoders run under it; the mix under rocprofv3 kernel tracing segfaults
# in a graph replay with or without the K/V-into-attention fusion.  Test the
# graph packet-capture path: the mix under the profiler with graphs launched
# node by node (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_mixdiag2; mkdir -p $O
cd /tmp
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mix -o run -- python3 $R/tools/podserver_once.py --mix yolos:20,llama-dec:8 --window 4 > $O/mix.log 2>&1 || { echo "mix failed"; grep -E "SIGSEGV|Aborted|Error" $O/mix.log | head -5; rm -rf $O/mix; exit 1; }
f=$(find $O/mix -name "*kernel_stats.csv" | head -1); cp $f $O/mix_kernel_stats.csv; rm -rf $O/mix
grep -h '^{' $O/mix.log | tail -1 | cut -c1-300
python3 - $O/mix_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{100*float(r["TotalDurationNs"])/tot:5.1f}% {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:8.1f}us {r["Name"][:90]}')
PY
