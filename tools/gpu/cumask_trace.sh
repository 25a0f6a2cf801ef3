# Kernel traces of 1 and 7 CU-mask process pods (bench.py --mode cumask) and
# their per-kernel durations vs dispatch gaps (tools/trace_gaps.py).
# usage (via gpurun): bash tools/gpu/cumask_trace.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cumask_trace}
mkdir -p $O
for N in 1 7; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$N -o run -- python3 $R/bench.py --mode cumask --pods-per-gpu $N --table "" --ref-pod-s 0 --extra-bf16-s 0 --steps 6 --warmup 2 --step-s 0.5 --json-out $O/bench$N.json > $O/t$N.log 2>&1 || { echo "trace $N failed"; tail -20 $O/t$N.log; exit 1; }
  cd $R && python3 tools/trace_gaps.py $O/t$N --json $O/gaps$N.json > /dev/null && rm -rf $O/t$N
  python3 -c "import json;d=json.load(open('$O/gaps$N.json'));print($N, d['gap_us'], list(d['per_kernel_us'].items())[:4])"
done
