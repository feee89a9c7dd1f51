set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | head -20 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
export AB_KINDS=sym,symk1 AB_SHAPES=100000x64,200000x30,500000x256
timeout -k 10 240 python -u scripts/gram_split_ab.py 3 > gpurun_out/sg_ab2.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/sg_ab2.log | cut -c1-250
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-2500
[ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/prof_r01c
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r01c/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_r01c/trace.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --warm-steps 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_r01c/f -o run --output-format csv -- $B > $R/gpurun_out/prof_r01c/f.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_r01c/w -o run --output-format csv -- $B > $R/gpurun_out/prof_r01c/w.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R && python3 scripts/pmc_summary.py gpurun_out/prof_r01c gram_sym
