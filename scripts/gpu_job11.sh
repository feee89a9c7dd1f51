set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | head -30 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-2500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
