set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_base; mkdir -p $O
timeout -k 10 200 python3 tools/podserver_once.py --tenants 28 --window 8 > $O/fleet.json 2> $O/fleet.err || { echo fleet failed; tail -5 $O/fleet.err; exit 1; }
cat $O/fleet.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('fleet', d['inf_per_s'], d['sclk_mhz'])"
timeout -k 10 300 python3 tools/ln_handoff_bench.py > $O/lnb.json 2> $O/lnb.err || { echo lnb failed; tail -5 $O/lnb.err; exit 1; }
tail -c 1500 $O/lnb.json
bash tools/gpu/pmc_fleet.sh r06_base/pmc_fleet 28
