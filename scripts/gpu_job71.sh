set -u
cd $GRAFT_REPO_ROOT
for t in 1 2 4; do
  DAL_FOREST_TPR=$t timeout -k 10 300 python -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b3_$t.log 2>&1; rc=$?
  echo "ilp8 tpr>=$t rc=$rc $(tail -1 gpurun_out/b3_$t.log | grep -o '"roofline_forest.*' | grep -o '"launch_ms": [0-9.]*') $(tail -1 gpurun_out/b3_$t.log | grep -o '"warm_selection_latency_ms": [0-9.]*')"
  [ $rc -eq 0 ] || exit $rc
done
