set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_LIBS=none AB_KNOBS=chunk=DAL_GRAM_CONTIG:0,nc5=DAL_GRAM_NC:5,nc10=DAL_GRAM_NC:10,nc56=DAL_GRAM_NC:56,ant0=DAL_GRAM_ANT:0 AB_SHAPES=100000x64,200000x64 AB_ROUNDS=5 timeout -k 10 300 python -u scripts/gram_ablate.py > gpurun_out/ab45.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ab45.log | cut -c1-200
