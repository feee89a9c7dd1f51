set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_LIBS=cred0 AB_SHAPES=100000x64,200000x64,284807x30,500000x256 AB_ROUNDS=5 timeout -k 10 300 python -u scripts/gram_ablate.py > gpurun_out/ab49.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ab49.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-300; tail -1 gpurun_out/bench_default.log | grep -o '"roofline.*' | cut -c1-300
