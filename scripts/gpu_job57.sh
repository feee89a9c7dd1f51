set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in 3 5 4; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/bench_config$c.log 2>&1; rc=$?
  echo "config $c rc=$rc"; tail -1 gpurun_out/bench_config$c.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -1 gpurun_out/prof_bench.log | cut -c1-300
