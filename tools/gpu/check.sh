# Standard GPU-box check: gpu tests, smoke, short 1-GPU bench, rocprofv3 kernel stats.
# usage (from the repo root, via gpurun): bash tools/gpu/check.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-check}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
if [ "${PROFILE:-1}" = 1 ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
  find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
  head -15 $O/kernel_stats.csv
fi
