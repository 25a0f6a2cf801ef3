# The last tree: a 1000-example GPU fuzz sweep (decode family included) and a 120 s
# soak of the default fleet (the reference demo's averaging window).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_soak_fuzz2; mkdir -p $O
timeout -k 10 900 python3 -u tools/fuzz_sweep.py --examples 1000 --out $O/fuzz.jsonl > $O/sweep.log 2>&1 || { echo sweep failed; tail -30 $O/sweep.log; exit 1; }
tail -1 $O/sweep.log
python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d['kind'], d['program']['name'], d['error'][:300].replace(chr(10),' '))
" $O/fuzz.jsonl | head -20
timeout -k 10 600 python -u bench.py --steps 200 --warmup 5 --table= --ref-pod-s 0 --extra-bf16-s 0 --json-out $O/soak.json > $O/soak.log 2>&1 || { echo soak failed; tail -20 $O/soak.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/soak.json'));print({k:d.get(k) for k in ('aggregate_inf_per_s','window_s','gpu_util_pct','rank0_sclk_mhz','matrix_pipe_util_pct')})"
