# Pod-server fleet kernel stats + x6 attention PMC + default bench, keeping
# gpurun_out small (only *stats* / counter CSVs; the copy-back limit is 64 MiB).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ps -o ps -- python3 $R/tools/podserver_once.py --tenants 28 --window 6 > $O/ps_prof.log 2>&1 || exit 1
find $O/prof_ps -type f ! -name "*kernel_stats*" -delete
tail -1 $O/ps_prof.log
cd $R
bash tools/gpu/pmc_attn.sh 8 x6n fp32,bf16 || exit 1
python tools/pmc_summary.py gpurun_out/pmc_attn_x6n_b8 --out $O/pmc_attn_x6n_b8.json > /dev/null || exit 1
rm -rf gpurun_out/pmc_attn_x6n_b8
timeout -k 10 600 python bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1 || exit 1
find $R/gpurun_out -type f -size +4M -print -delete
du -sh $R/gpurun_out
