# One GPU-box session: pod-server GPU tests first (fail fast), the whole GPU
# suite, smoke(), then the default bench (server mode) as JSON.
# usage (via gpurun, from the repo root): bash tools/gpu/session.sh <tag> [bench args...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-session}; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_podserver_gpu.py -x -v --timeout 200 --timeout-method thread > $O/podserver_gpu.log 2>&1 || { echo podserver gpu tests failed; tail -40 $O/podserver_gpu.log; exit 1; }
tail -2 $O/podserver_gpu.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { echo gpu tests failed; tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 700 python bench.py --json-out $O/bench.json "$@" > $O/bench.log 2>&1 || { echo bench failed; tail -30 $O/bench.log; exit 1; }
python - <<PY
import json; d=json.load(open("$O/bench.json"))
print({k: d.get(k) for k in ["value","vs_baseline","aggregate_inf_per_s","single_pod_inf_per_s","aggregate_vs_single_pod","matrix_pipe_util_pct","rank0_sclk_mhz","gpu_util_pct"]})
print("bf16", (d.get("bf16_gfx950_kernels") or {}).get("inf_per_s"))
for r in d.get("latency_table") or []: print(r)
PY
