set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_KINDS=sym0,sym timeout -k 10 240 python -u scripts/gram_split_ab.py 3 > gpurun_out/split_ab5.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/split_ab5.log
