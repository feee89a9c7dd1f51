set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python -u scripts/host_overhead.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-300; tail -1 gpurun_out/bench_default.log | grep -o '"roofline.*' | cut -c1-300
