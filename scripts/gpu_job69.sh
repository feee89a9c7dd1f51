set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for c in 3 2; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/bench_config$c.log 2>&1; rc=$?
  echo "config $c rc=$rc $(tail -1 gpurun_out/bench_config$c.log | grep -o '"ms_per_step": [0-9.]*') $(tail -1 gpurun_out/bench_config$c.log | grep -o '"launch_ms": [0-9.]*' | head -1) $(tail -1 gpurun_out/bench_config$c.log | grep -o '"warm_selection_latency_ms": [0-9.]*')"
  [ $rc -eq 0 ] || exit $rc
done
