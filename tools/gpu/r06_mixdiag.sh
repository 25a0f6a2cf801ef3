# The YOLOS + decoders mix segfaulted in a graph replay under rocprofv3 kernel
# tracing (r06_final3). Narrow it: the mix without the profiler, 8 decoders
# under the profiler, the mix under the profiler without the K/V-write-into-
# attention fusion, then the default mix under the profiler again.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_mixdiag; mkdir -p $O
timeout -k 10 300 python3 tools/podserver_once.py --mix yolos:20,llama-dec:8 --window 8 > $O/mix_noprof.json 2> $O/mix_noprof.err || { echo "mix (no profiler) failed"; tail -8 $O/mix_noprof.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('noprof', d['inf_per_s'], d['decode_token_latency_ms'], {k: v['inf_per_s'] for k, v in d['per_kind'].items()}, d['sclk_mhz'])" $O/mix_noprof.json
cd /tmp
prof() {  # tag, env assignments..., then the mix
  tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 $R/tools/podserver_once.py --mix $1 --window 4 > $O/$tag.log 2>&1 || { echo "$tag failed"; grep -E "SIGSEGV|Aborted|Error" $O/$tag.log | head -5; rm -rf $O/$tag; return 1; }
  f=$(find $O/$tag -name "*kernel_stats.csv" | head -1); cp $f $O/${tag}_kernel_stats.csv; rm -rf $O/$tag
  echo "$tag ok"
}
prof dec8 llama-dec:8 || exit 1
NOS_AMD_SKIP_PASSES=kv_into_attention prof mix_nofresh yolos:20,llama-dec:8 || exit 1
prof mix yolos:20,llama-dec:8 || exit 1
