set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2 -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --warm-steps 0 --no-cpu-baseline > $R/gpurun_out/prof_c2.log 2>&1; rc=$?; echo "prof rc=$rc"; tail -1 $R/gpurun_out/prof_c2.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_c2 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --warm-steps 0 --no-cpu-baseline > $R/gpurun_out/pmc_fetch_c2.log 2>&1; rc=$?; echo "pmc fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_c2 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --warm-steps 0 --no-cpu-baseline > $R/gpurun_out/pmc_write_c2.log 2>&1; rc=$?; echo "pmc write rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 400 python -u bench.py --config 4 --steps 2 --warmup 1 --warm-steps 2 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1; rc=$?; echo "bench c4 rc=$rc"; tail -1 gpurun_out/bench_c4.log | cut -c1-1500
