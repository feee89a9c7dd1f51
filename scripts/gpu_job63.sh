set -u
cd $GRAFT_REPO_ROOT
for b in 16384 32768 65536 98304 135168; do
  DAL_FOREST_TILE_BYTES=$b timeout -k 10 300 python -u bench.py --config 4 --steps 1 --warmup 1 --warm-steps 10 --no-cpu-baseline > gpurun_out/b4_$b.log 2>&1; rc=$?
  echo "tile<=$b rc=$rc $(tail -1 gpurun_out/b4_$b.log | grep -o '"roofline_forest.*' | grep -o '"launch_ms": [0-9.]*') $(tail -1 gpurun_out/b4_$b.log | grep -o '"warm_selection_latency_ms": [0-9.]*')"
  [ $rc -eq 0 ] || exit $rc
done
