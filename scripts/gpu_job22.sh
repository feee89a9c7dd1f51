set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_LIBS=prev AB_KNOBS=two=DAL_GRAM_ONE:0 timeout -k 10 200 python -u scripts/gram_ablate.py > gpurun_out/ablate2.log 2>&1; rc=$?
echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate2.log
