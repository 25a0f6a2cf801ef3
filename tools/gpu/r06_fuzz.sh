# Fuzz sweep (every failure recorded), then the fuzz + decode GPU tests.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_fuzz; mkdir -p $O
timeout -k 10 600 python3 -u tools/fuzz_sweep.py --examples 400 --out $O/fuzz.jsonl > $O/sweep.log 2>&1 || { echo sweep failed; tail -30 $O/sweep.log; exit 1; }
tail -1 $O/sweep.log
python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d['kind'], d['program']['name'], d['error'][:400].replace(chr(10),' '))
" $O/fuzz.jsonl
timeout -k 10 900 python -u -m pytest tests/test_decode_gpu.py tests/test_program_fuzz_gpu.py -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
