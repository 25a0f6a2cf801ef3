# Round-3 session-2 GPU pass: x6 scalar-split A/B, pod-server fleet kernel
# trace, default bench.  bash tools/gpu/r03_s2.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s2
mkdir -p $O
bash tools/gpu/attn_dma_ab.sh x6scalar x6scalar || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ps -o ps -- python3 $R/tools/podserver_once.py --tenants 28 --window 6 > $O/ps_prof.log 2>&1 || exit 1
tail -1 $O/ps_prof.log
cd $R
timeout -k 10 600 python bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1 || exit 1
python -c "import json;d=json.load(open('$O/bench_default.json'));print({k:d[k] for k in ['value','vs_baseline','aggregate_inf_per_s','single_pod_inf_per_s','rank0_sclk_mhz']}); [print(r) for r in d['latency_table']]"
