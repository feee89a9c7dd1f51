set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/sharded_overhead.py 20 > gpurun_out/sharded_overhead.log 2>&1; rc=$?
echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/sharded_overhead.log | tail -8
