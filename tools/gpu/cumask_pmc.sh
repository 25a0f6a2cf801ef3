# Round 5: where a CU-mask slice's time goes under
# contention.  One masked YOLOS pod (32 CUs = a 36 GB slice, slice-sized
# persistent grids) under rocprofv3 PMC passes -- HBM bytes per inference
# (FETCH_SIZE / WRITE_SIZE), L2 hit rate, busy cycles -- then the bench's
# latency table, whose rows now carry amd-smi UMC (HBM controller) activity.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_cumask
mkdir -p $O
cd /tmp
i=0
for CNT in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $O/pass$i -o run -- python3 $R/tools/pod_once.py --memory-fraction 0.125 --cu-mask 0xffffffff --iters 10 > $O/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
done
cd $R
python3 tools/pmc_summary.py $O --out $O/summary.json > $O/summary.log 2>&1 || { tail -5 $O/summary.log; }
rm -rf $O/pass1 $O/pass2 $O/pass3
timeout -k 10 150 python3 tools/pod_once.py --memory-fraction 0.125 --cu-mask 0xffffffff --iters 30 > $O/solo_masked.log 2>&1; tail -1 $O/solo_masked.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --table-modes cumask,shared --extra-bf16-s 0 --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print([(r['mode'],r['pods'],r['inf_per_s'],r.get('latency_vs_solo_at_solo_clock'),r.get('umc_util_pct')) for r in d['latency_table']])"
