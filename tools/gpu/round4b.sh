# Pod-server GPU tests, fleet layout A/B (tools/gpu/fleet_ab2.sh), quota run.
# usage (via gpurun): bash tools/gpu/round4b.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4b}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_podserver_gpu.py -x -q --timeout 200 --timeout-method thread > $O/podserver_gpu.log 2>&1 || { echo podserver gpu tests failed; tail -40 $O/podserver_gpu.log; exit 1; }
tail -1 $O/podserver_gpu.log
bash tools/gpu/fleet_ab2.sh ${1:-r4b}_fab || exit 1
timeout -k 10 600 python bench.py --quota --json-out $O/quota.json 2>&1 | tee $O/quota.log || { echo quota failed; exit 1; }
