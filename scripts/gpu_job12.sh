set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 240 python -u scripts/gram_split_ab.py 3 > gpurun_out/split_ab.log 2>&1; rc=$?
echo "ab rc=$rc"; cat gpurun_out/split_ab.log | grep -v amdgpu.ids
