# One decoder (generate loop) under kernel tracing: per-kernel time per step by
# kernel and grid size (tools/decode_gaps.py); traces deleted.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_dec1prof2; mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/tools/podserver_once.py --mix llama-dec:1 --window 3 --gen-chunk 64 > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; rm -rf $O/prof; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
head -1 $f > $O/trace_header.txt
python3 $R/tools/decode_gaps.py $f --tail 5000 > $O/gaps.json && rm -rf $O/prof
cat $O/gaps.json
