# BASELINE config 5 composed on one MI355X: the shared-pool run (CU-masked
# trainer + partition pods as pod-server tenants + team-a waves + preemption)
# and the split-policy run (team-b on an isolated CU pool, latency alone vs
# beside team-a's bursts).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_config5; mkdir -p $O
timeout -k 10 900 python -u bench.py --quota --composed --json-out $O/composed.json > $O/composed.log 2>&1 || { echo composed failed; tail -30 $O/composed.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/composed.json'))
print({k: v for k, v in d.items() if not isinstance(v, (dict, list))})
for k, v in d.items():
    if isinstance(v, dict) and k.startswith('phase'): print(k, {a: b for a, b in v.items() if not isinstance(b, (dict, list))})
"
timeout -k 10 900 python -u bench.py --quota --composed --isolate-team-b --json-out $O/isolated.json > $O/isolated.log 2>&1 || { echo isolated failed; tail -30 $O/isolated.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/isolated.json'))
print({k: v for k, v in d.items() if not isinstance(v, (dict, list))})
for k, v in d.items():
    if isinstance(v, dict): print(k, {a: b for a, b in v.items() if not isinstance(b, (dict, list))})
"
