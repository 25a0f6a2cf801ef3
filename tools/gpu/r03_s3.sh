# Round-3 session-2 GPU pass 2: GPU tests + smoke on the adopted kernels,
# pod-server fleet kernel stats (trace files dropped: the copy-back limit is
# 64 MiB), default bench.  bash tools/gpu/r03_s3.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || exit 1
tail -1 $O/gputests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ps -o ps -- python3 $R/tools/podserver_once.py --tenants 28 --window 6 > $O/ps_prof.log 2>&1 || exit 1
find $O/prof_ps -name "*kernel_trace*" -delete
tail -1 $O/ps_prof.log
cd $R
timeout -k 10 600 python bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1 || exit 1
python -c "import json;d=json.load(open('$O/bench_default.json'));print({k:d[k] for k in ['value','vs_baseline','aggregate_inf_per_s','single_pod_inf_per_s','rank0_sclk_mhz']}); [print(r) for r in d['latency_table']]"
du -sh $O
