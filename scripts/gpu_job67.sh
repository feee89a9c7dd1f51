set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config 3 > gpurun_out/bench_config3.log 2>&1; rc=$?
echo "config 3 rc=$rc $(tail -1 gpurun_out/bench_config3.log | cut -c1-250)"; tail -1 gpurun_out/bench_config3.log | grep -o '"frac": [0-9.]*' | head -1
