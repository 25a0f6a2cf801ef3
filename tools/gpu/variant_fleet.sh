# Fleet and GEMM-kernel A/B of kernel variants built by tools/build_variant.py
# (build/variants/<name>/libnos_hip.so; "base" = the in-tree library).
# usage (via gpurun): bash tools/gpu/variant_fleet.sh <tag> <variant> [<variant> ...]
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
mkdir -p $O
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then unset NOS_AMD_HIP_LIB; else export NOS_AMD_HIP_LIB=$GRAFT_REPO_ROOT/build/variants/$v/libnos_hip.so; fi
    if [ $r = 1 ]; then
      timeout -k 10 200 python tools/kernel_bench.py --only gemm --dtype fp32 --f32-math x6 --x6-tile 5 --batch 1 --iters 20 --rounds 2 --out $O/kb_$v.json > $O/kb_$v.log 2>&1 || { echo "kernel_bench $v failed"; tail -20 $O/kb_$v.log; exit 1; }
    fi
    timeout -k 10 240 python -u tools/podserver_once.py --tenants 28 --window 8 > $O/fleet_${v}_r$r.json 2> $O/fleet_${v}_r$r.err || { echo "fleet $v failed"; tail -20 $O/fleet_${v}_r$r.err; exit 1; }
    echo "$v r$r $(cat $O/fleet_${v}_r$r.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["inf_per_s"], d["sclk_mhz"])')"
  done
done
unset NOS_AMD_HIP_LIB
python - $O "$@" <<'PY'
import json,sys
O=sys.argv[1]
for v in sys.argv[2:]:
    a=json.load(open(f"{O}/kb_{v}.json"))
    print(v, {k.replace("_us",""): round(a[k],1) for k in a if k.endswith("_us") and "torch" not in k})
PY
