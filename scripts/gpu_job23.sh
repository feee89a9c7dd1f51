set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|error" gpurun_out/pytest_gpu.log | head -30 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-1200
[ $rc -eq 0 ] || exit $rc
DAL_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_gloo2.log 2>&1; rc=$?; echo "gloo2 rc=$rc"; grep metric gpurun_out/bench_gloo2.log | cut -c1-600
