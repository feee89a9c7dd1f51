set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | head -20 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-700
[ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/prof_r01d
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r01d/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_r01d/trace.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R
DAL_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_gloo2.log 2>&1; rc=$?; echo "gloo2 rc=$rc"; grep metric gpurun_out/bench_gloo2.log | cut -c1-200
