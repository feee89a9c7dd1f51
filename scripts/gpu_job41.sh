set -u
R=$GRAFT_REPO_ROOT
cd $R
export AB_KINDS=sym,split AB_SHAPES=284807x30,200000x30
timeout -k 10 240 python -u scripts/gram_split_ab.py 3 > gpurun_out/sg_ab5.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/sg_ab5.log | cut -c1-200
