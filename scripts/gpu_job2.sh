set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 480 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log | cut -c1-300
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1; rc=$?; echo "bench c2 rc=$rc"; tail -1 gpurun_out/bench_c2.log | cut -c1-2000
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2b -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --warm-steps 0 --no-cpu-baseline > $R/gpurun_out/prof_c2b.log 2>&1; rc=$?; echo "prof rc=$rc"
head -8 $R/gpurun_out/prof_c2b/run_kernel_stats.csv | cut -c1-200
[ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 400 python -u bench.py --config 4 --steps 2 --warmup 1 --warm-steps 2 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1; rc=$?; echo "bench c4 rc=$rc"; tail -1 gpurun_out/bench_c4.log | cut -c1-1500
