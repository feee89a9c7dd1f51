set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_LIBS=abl1,abl2,abl3,abl4,abl5 AB_SHAPES=100000x64,200000x64,284807x30 AB_ROUNDS=5 timeout -k 10 240 python -u scripts/gram_ablate.py > gpurun_out/ablate4.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate4.log | cut -c1-200
