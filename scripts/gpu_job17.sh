set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|error" gpurun_out/pytest_gpu.log | head -30 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-3000
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1; rc=$?; echo "bench c3 rc=$rc"; tail -1 gpurun_out/bench_c3.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2 -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_c2.log 2>&1; rc=$?; echo "prof rc=$rc"
