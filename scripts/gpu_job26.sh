set -u
R=$GRAFT_REPO_ROOT
cd $R
export AB_KINDS=symk1,symk2 AB_SHAPES=100000x64,200000x64,300000x128,500000x256
timeout -k 10 240 python -u scripts/gram_split_ab.py 3 > gpurun_out/sg_ab3.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/sg_ab3.log | cut -c1-250
