set -u
cd $GRAFT_REPO_ROOT
for b in 4112 8224 16448; do
  DAL_FOREST_TILE_BYTES=$b timeout -k 10 300 python -u bench.py --config 4 --steps 1 --warmup 1 --warm-steps 10 --no-cpu-baseline > gpurun_out/b4_$b.log 2>&1; rc=$?
  echo "cfg4 tile<=$b rc=$rc $(tail -1 gpurun_out/b4_$b.log | grep -o '"roofline_forest.*' | grep -o '"launch_ms": [0-9.]*') $(tail -1 gpurun_out/b4_$b.log | grep -o '"warm_selection_latency_ms": [0-9.]*')"
  [ $rc -eq 0 ] || exit $rc
done
for b in 4160 8320 16640 33280; do
  DAL_FOREST_TILE_BYTES=$b timeout -k 10 300 python -u bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b2_$b.log 2>&1; rc=$?
  echo "cfg2 tile<=$b rc=$rc $(tail -1 gpurun_out/b2_$b.log | grep -o '"roofline_forest.*' | grep -o '"launch_ms": [0-9.]*') $(tail -1 gpurun_out/b2_$b.log | grep -o '"warm_selection_latency_ms": [0-9.]*')"
  [ $rc -eq 0 ] || exit $rc
done
for b in 3968 7936 15872 31744; do
  DAL_FOREST_TILE_BYTES=$b timeout -k 10 300 python -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b3_$b.log 2>&1; rc=$?
  echo "cfg3 tile<=$b rc=$rc $(tail -1 gpurun_out/b3_$b.log | grep -o '"roofline_forest.*' | grep -o '"launch_ms": [0-9.]*') $(tail -1 gpurun_out/b3_$b.log | grep -o '"warm_selection_latency_ms": [0-9.]*')"
  [ $rc -eq 0 ] || exit $rc
done
