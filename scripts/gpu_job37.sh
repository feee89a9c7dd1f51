set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_ROUNDS=9 AB_SHAPES=100000x64,200000x64 AB_LIBS=none AB_KNOBS=nt=DAL_GRAM_ANT:1 timeout -k 10 300 python -u scripts/gram_ablate.py > gpurun_out/ablate8.log 2>&1; rc=$?
echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate8.log
