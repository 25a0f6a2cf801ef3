# The reference demo's latency-vs-pods table (1/3/5/7 pods per GPU) on one MI355X:
# YOLOS-small pods as separate processes (the real deployment) and as in-process
# CU-masked streams (bench.py's data plane), CU-mask slices vs unmasked sharing.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-demo_table}
mkdir -p $O
timeout -k 10 500 python tools/pod_procs.py --pods 1,3,5,7 --modes shared,cumask --iters 60 --out $O/pod_procs.json > $O/pod_procs.log 2>&1 || { tail -20 $O/pod_procs.log; exit 1; }
cat $O/pod_procs.log | grep '^{' || true
timeout -k 10 300 python tools/tenant_sweep.py --pods 1,3,5,7 --modes shared,cumask --steps 40 --out $O/sweep.json > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
grep '^{' $O/sweep.log || true
