set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python -u scripts/gram_ablate.py > gpurun_out/ablate.log 2>&1; rc=$?
echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate.log
