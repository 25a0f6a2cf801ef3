# GPU test suite, then the config-5 quota run (bench.py --quota) and the
# CU-mask 1 vs 7 pod kernel traces.  usage (via gpurun): bash tools/gpu/quota_cumask.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-qc}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { echo gpu tests failed; tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 600 python bench.py --quota --json-out $O/quota.json 2>&1 | tee $O/quota.log || { echo quota failed; exit 1; }
python3 -c "import json;d=json.load(open('$O/quota.json'));print(json.dumps({k:d[k] for k in ('phase_a','phase_b','concurrent_tenants')}))"
bash tools/gpu/cumask_trace.sh ${1:-qc}_trace
