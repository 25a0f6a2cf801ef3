# Column-split GEMM operands (training / matmul) tests, then the attention
# occupancy A/B, decode profiles and the reserved-CU queue test.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_cols; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train_ops_gpu.py tests/test_training_tenants_gpu.py tests/test_tenant_programs_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo col tests failed; grep -E "Error|assert|FAILED|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/train_once.py --seq 2048 --steps 6 --small 1 > $O/train.json 2> $O/train.err || { echo train_once failed; tail -5 $O/train.err; exit 1; }
cat $O/train.json
bash tools/gpu/r06_combo2.sh
