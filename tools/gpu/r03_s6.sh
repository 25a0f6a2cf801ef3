# Pod-server fleet kernel stats (CSV, trace dropped) + x6 GEMM PMC passes.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s6
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ps -o ps -- python3 $R/tools/podserver_once.py --tenants 28 --window 6 > $O/ps_prof.log 2>&1 || exit 1
find $O/prof_ps -type f ! -name "*stats*" -delete
find $O/prof_ps -type f
cd $R
PMC_OUT=s6/pmc_gemm_f32 bash tools/gpu/pmc_gemm_f32.sh || exit 1
python tools/pmc_summary.py gpurun_out/s6/pmc_gemm_f32 --out $O/pmc_gemm_f32.json > /dev/null || exit 1
rm -rf gpurun_out/s6/pmc_gemm_f32
find $R/gpurun_out -type f -size +4M -print -delete
du -sh $R/gpurun_out
