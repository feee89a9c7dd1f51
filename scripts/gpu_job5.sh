set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?; echo "bench c5 rc=$rc"; tail -2 gpurun_out/bench_c5.log | cut -c1-2500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1; rc=$?; echo "bench c3 rc=$rc"; tail -1 gpurun_out/bench_c3.log | cut -c1-2500
[ $rc -eq 0 ] || exit $rc
DAL_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --warm-steps 2 > gpurun_out/bench_c2_p2_gloo.log 2>&1; rc=$?; echo "bench p2 gloo rc=$rc"; tail -3 gpurun_out/bench_c2_p2_gloo.log | cut -c1-2500
[ $rc -eq 0 ] || exit $rc
DAL_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config 5 --steps 2 --warmup 1 > gpurun_out/bench_c5_p2_gloo.log 2>&1; rc=$?; echo "bench c5 p2 gloo rc=$rc"; tail -3 gpurun_out/bench_c5_p2_gloo.log | cut -c1-2500
