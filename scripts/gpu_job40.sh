set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/prof_r01e
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r01e/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_r01e/trace.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --warm-steps 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_r01e/f -o run --output-format csv -- $B > $R/gpurun_out/prof_r01e/f.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_r01e/w -o run --output-format csv -- $B > $R/gpurun_out/prof_r01e/w.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R && python3 scripts/pmc_summary.py gpurun_out/prof_r01e gram_sym2
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-300
