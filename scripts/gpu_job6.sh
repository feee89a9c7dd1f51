set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | head -30 | cut -c1-300
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1; rc=$?; echo "bench c2 rc=$rc"; tail -1 gpurun_out/bench_c2.log | cut -c1-3000
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_job5.sh
