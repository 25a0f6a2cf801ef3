# End-of-session check of the tree as committed: GPU tests, smoke, default bench.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/final
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || exit 1
tail -1 $O/gputests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || exit 1
python -c "import json;d=json.load(open('$O/bench.json'));print({k:d[k] for k in ['value','vs_baseline','aggregate_inf_per_s','single_pod_inf_per_s','rank0_sclk_mhz']}, d['bf16_gfx950_kernels']['inf_per_s'])"
