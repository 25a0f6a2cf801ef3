set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r32
mkdir -p $O
V=build/variants/$1/libnos_hip.so
NOS_AMD_HIP_LIB=$V timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "attention or yolos" > $O/pytest_$1.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_$1.log
if [ $rc -ne 0 ]; then exit $rc; fi
for B in 1 8; do
timeout -k 10 100 python tools/kernel_bench.py --only attn --batch $B --iters 20 --out $O/base_b$B.json > /dev/null 2>&1 && \
NOS_AMD_HIP_LIB=$V timeout -k 10 100 python tools/kernel_bench.py --only attn --batch $B --iters 20 --out $O/$1_b$B.json > /dev/null 2>&1 || exit 1
done
NOS_AMD_HIP_LIB=$V timeout -k 10 300 python bench.py --steps 20 > $O/bench_$1.log 2>&1
echo rc=$?
