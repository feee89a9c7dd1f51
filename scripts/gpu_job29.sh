set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1; rc=$?; echo "c3 rc=$rc"; tail -1 gpurun_out/bench_c3.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config 4 --steps 2 --warmup 1 --warm-steps 2 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1; rc=$?; echo "c4 rc=$rc"; tail -1 gpurun_out/bench_c4.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?; echo "c5 rc=$rc"; tail -1 gpurun_out/bench_c5.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
DAL_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_gloo2.log 2>&1; rc=$?; echo "gloo2 rc=$rc"; grep metric gpurun_out/bench_gloo2.log | cut -c1-300
