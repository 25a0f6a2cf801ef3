set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r28
mkdir -p $O
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/kernel_bench.py --only gemm --batch 8 --iters 20 --out $O/gemm_b8.json > $O/gemm_b8.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 > $O/bench.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -- python3 $GRAFT_REPO_ROOT/tools/kernel_bench.py --only attn,gemm --batch 8 --iters 3 > $O/pmc2.log 2>&1
echo rc=$?
