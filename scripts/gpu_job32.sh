set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_ROUNDS=9 AB_SHAPES=100000x64,200000x64 AB_LIBS=none AB_KNOBS=nc5=DAL_GRAM_NC:5,nc7=DAL_GRAM_NC:7,nc10=DAL_GRAM_NC:10,nc14=DAL_GRAM_NC:14,nc20=DAL_GRAM_NC:20 timeout -k 10 300 python -u scripts/gram_ablate.py > gpurun_out/ablate5.log 2>&1; rc=$?
echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate5.log
AB_ROUNDS=4 AB_SHAPES=500000x256 AB_LIBS=none AB_KNOBS=nc4=DAL_GRAM_NC:4,nc6=DAL_GRAM_NC:6,nc8=DAL_GRAM_NC:8,nc16=DAL_GRAM_NC:16 timeout -k 10 300 python -u scripts/gram_ablate.py > gpurun_out/ablate6.log 2>&1; rc=$?
echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate6.log
