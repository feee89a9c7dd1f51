set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_ROUNDS=9 AB_SHAPES=100000x64 AB_LIBS=none AB_KNOBS=k1=DAL_GRAM_SYM:1,nc8=DAL_GRAM_NC:8,nc14=DAL_GRAM_NC:14,nc20=DAL_GRAM_NC:20,nc28=DAL_GRAM_NC:28,nc40=DAL_GRAM_NC:40,nc56=DAL_GRAM_NC:56 timeout -k 10 300 python -u scripts/gram_ablate.py > gpurun_out/ablate7.log 2>&1; rc=$?
echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate7.log
