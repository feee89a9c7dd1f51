set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_maxcos.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | head -30 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5 -o run --output-format csv -- python3 $R/bench.py --config 5 --steps 3 --warmup 1 > $R/gpurun_out/prof_c5.log 2>&1; rc=$?; echo "prof c5 rc=$rc"; tail -1 $R/gpurun_out/prof_c5.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2 -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --warm-steps 0 --no-cpu-baseline > $R/gpurun_out/prof_c2.log 2>&1; rc=$?; echo "prof c2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_c2 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --warm-steps 0 --no-cpu-baseline > $R/gpurun_out/pmc_fetch_c2.log 2>&1; rc=$?; echo "pmc fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_c2 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --warm-steps 0 --no-cpu-baseline > $R/gpurun_out/pmc_write_c2.log 2>&1; rc=$?; echo "pmc write rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?; echo "bench c5 rc=$rc"; tail -1 gpurun_out/bench_c5.log | cut -c1-2500
