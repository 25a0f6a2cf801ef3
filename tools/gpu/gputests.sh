# GPU tests: the named files first (-x, verbose), then the whole -m gpu suite.
# usage (GPU box, repo root): bash tools/gpu/gputests.sh <tag> [test files...]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-gputests}; shift; mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread > $O/first.log 2>&1 || { echo first failed; grep -E "FAILED|Error|assert|passed|failed" $O/first.log | head -40; tail -30 $O/first.log; exit 1; }
  tail -2 $O/first.log
fi
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/all.log 2>&1 || { echo suite failed; grep -E "FAILED|Error" $O/all.log | head -30; tail -30 $O/all.log; exit 1; }
tail -2 $O/all.log
