# Config 5 split-policy (isolated team-b) run, then the decode latency A/B.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_config5; mkdir -p $O
timeout -k 10 500 python -u bench.py --quota --composed --isolate-team-b --json-out $O/isolated.json > $O/isolated.log 2>&1 || { echo isolated failed; grep -v "tenants ready" $O/isolated.log | tail -20; exit 1; }
python3 -c "
import json; d=json.load(open('$O/isolated.json'))
print({k: v for k, v in d.items() if not isinstance(v, (dict, list))})
for k, v in d.items():
    if isinstance(v, dict) and k.startswith('phase'): print(k, {a: b for a, b in v.items() if a in ('ok', 'seconds', 'gpu_util_pct', 'latency', 'trainer')})
"
bash tools/gpu/r06_lat.sh
