set -u
cd $GRAFT_REPO_ROOT
for c in 2 3 4; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/bench_config$c.log 2>&1; rc=$?
  echo "config $c rc=$rc"; tail -1 gpurun_out/bench_config$c.log | grep -o '"roofline_forest.*' | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
