# rocprofv3 PMC passes over the h3 GEMM (2x2 / 4x1), the LN row split and h3 attention
# (tools/h3_pmc_once.py).  usage (GPU box, repo root): bash tools/gpu/pmc_h3.sh <tag>
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${1:-pmc_h3}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CNT in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/pass$i -o run -- python3 $R/tools/h3_pmc_once.py > $OUT/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pass$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT --out $OUT/summary.json && rm -rf $OUT/pass1 $OUT/pass2 $OUT/pass3 && python3 - $OUT/summary.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
for k,v in d.items():
    if isinstance(v,dict) and "derived" in v: print(k[:90], {a: round(b,2) for a,b in v["derived"].items()})
PY
