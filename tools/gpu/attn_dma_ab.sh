# A/B of the in-tree kernels ("new") against variant libraries under
# build/variants/<name>/libnos_hip.so: kernel numerics, attention throughput,
# fleet bench.  bash tools/gpu/attn_dma_ab.sh <out-tag> <variant> [<variant> ...]
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift
TAGS="$* new"
mkdir -p $O
lib() { [ "$1" = new ] || echo build/variants/$1/libnos_hip.so; }
for tag in $TAGS; do
  NOS_AMD_HIP_LIB=$(lib $tag) timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
    --timeout-method thread > $O/kernels_$tag.log 2>&1 || exit 1
  echo "$tag: $(tail -1 $O/kernels_$tag.log)"
done
for R in 1 2; do for tag in $TAGS; do
  for v in "--dtype fp32 --variant x6" "--dtype fp32 --variant x6n" "--dtype fp32 --variant auto" "--dtype bf16"; do
    NOS_AMD_HIP_LIB=$(lib $tag) timeout -k 10 120 python tools/attn_bench.py $v --batches 1,8 | sed "s/^{/{\"lib\": \"$tag\", /" >> $O/attn.jsonl 2>>$O/err.log || exit 1
  done
done; done
python - $O/attn.jsonl <<'PY'
import json, sys, collections
best = collections.defaultdict(dict)
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    k = (d["dtype"], d["variant"], d["B"])
    best[k][d["lib"]] = min(best[k].get(d["lib"], 1e99), d["us"])
for k, v in sorted(best.items()):
    print(k, v)
PY
for tag in $TAGS; do
  NOS_AMD_HIP_LIB=$(lib $tag) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ref-pod-s 0 --table '' --extra-bf16-s 5 \
    --json-out $O/bench_${tag}.json > /dev/null 2>>$O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/bench_${tag}.json'));print('$tag', d['value'], d['aggregate_inf_per_s'], d['rank0_sclk_mhz'], d['bf16_gfx950_kernels']['inf_per_s'])"
done
