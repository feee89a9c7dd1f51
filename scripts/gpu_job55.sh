set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/tl -o tl --output-format csv -- python3 scripts/step_timeline.py > gpurun_out/tl.log 2>&1; rc=$?
[ $rc -eq 0 ] || exit $rc
python3 scripts/step_timeline.py --analyse gpurun_out/tl > gpurun_out/tl_summary.txt; cat gpurun_out/tl_summary.txt
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-400; tail -1 gpurun_out/bench_default.log | grep -o '"warm_sel.*' | cut -c1-120
