set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config 4 --steps 1 --warmup 1 --warm-steps 10 --no-cpu-baseline > gpurun_out/bp_4.log 2>&1; rc=$?
echo "cfg4 rc=$rc $(tail -1 gpurun_out/bp_4.log | grep -o '"roofline_forest.*' | grep -o '"launch_ms": [0-9.]*') $(tail -1 gpurun_out/bp_4.log | grep -o '"warm_selection_latency_ms": [0-9.]*')"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-300; tail -1 gpurun_out/bench_default.log | grep -o '"roofline_forest.*' | grep -o '"launch_ms": [0-9.]*'
