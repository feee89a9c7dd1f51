set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for c in 3 4 2; do
for p in 0 1; do
  DAL_FOREST_PERSIST=$p timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 --warm-steps 10 --no-cpu-baseline > gpurun_out/bp_$c$p.log 2>&1; rc=$?
  echo "cfg$c persist=$p rc=$rc $(tail -1 gpurun_out/bp_$c$p.log | grep -o '"roofline_forest.*' | grep -o '"launch_ms": [0-9.]*') $(tail -1 gpurun_out/bp_$c$p.log | grep -o '"warm_selection_latency_ms": [0-9.]*')"
  [ $rc -eq 0 ] || exit $rc
done
done
