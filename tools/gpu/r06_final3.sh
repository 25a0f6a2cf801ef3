# The training fuzz, then the round-6 final check.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_final3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_training_fuzz_gpu.py -q --timeout 500 --timeout-method thread > $O/train_fuzz.log 2>&1 || { echo training fuzz failed; grep -E "Error|assert|FAILED|failed|Falsifying" $O/train_fuzz.log | head -30; tail -5 $O/train_fuzz.log; exit 1; }
tail -1 $O/train_fuzz.log
bash tools/gpu/r06_final.sh r06_final3
