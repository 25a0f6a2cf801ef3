set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest14.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest14.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench14.log 2>&1 && \
timeout -k 10 300 python bench.py --mode cumask > gpurun_out/bench14c.log 2>&1 && \
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke14.log 2>&1
echo rc=$?
