set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_LIBS=none AB_KNOBS=abl1=DAL_GRAM_ABL:1,abl2=DAL_GRAM_ABL:2,abl3=DAL_GRAM_ABL:3,k1=DAL_GRAM_SYM:1 timeout -k 10 200 python -u scripts/gram_ablate.py > gpurun_out/ablate3.log 2>&1; rc=$?
echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate3.log
