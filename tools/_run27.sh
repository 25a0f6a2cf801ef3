set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r27
mkdir -p $O
cd /tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc1 -- python3 $GRAFT_REPO_ROOT/tools/kernel_bench.py --only attn --batch 8 --iters 5 > $O/pmc1.log 2>&1
echo rc=$?
