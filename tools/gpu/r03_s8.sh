# x6 attention without the padding-row memset: kernel tests (incl. NaN in the
# padding rows), then the 28-tenant fleet in-tree vs build/variants/prev.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/kernels.log 2>&1 || exit 1
tail -1 $O/kernels.log
for round in 1 2; do for tag in new prev; do
  L=; [ $tag = prev ] && L=build/variants/prev/libnos_hip.so
  NOS_AMD_HIP_LIB=$L timeout -k 10 120 python tools/podserver_once.py --tenants 28 --window 8 2>>$O/err.log \
    | sed "s/^{/{\"lib\": \"$tag\", \"round\": $round, /" >> $O/fleet.jsonl || exit 1
done; done
python -c "
import json
for l in open('$O/fleet.jsonl'): d=json.loads(l); print(d['lib'], d['round'], d['inf_per_s'])"
