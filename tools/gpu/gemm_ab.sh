# A/B of the GEMM epilogue implementations: numerics, per-kernel time, bench.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-gemm_ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "linear or yolos" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for B in 1 8; do
  timeout -k 10 200 python tools/kernel_bench.py --only gemm --batch $B --iters 20 --rounds 3 --impls register,lds --out $O/kb_b$B.json > /dev/null 2> $O/kb_b$B.err || { tail $O/kb_b$B.err; exit 1; }
  cat $O/kb_b$B.json | tr -d '\n'; echo
done
for I in register lds register lds; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --gemm-impl $I > $O/bench_$I.json 2>>$O/bench.err || { tail $O/bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$I.json'));print('$I',d['value'],d['ms_per_step'])"
done
