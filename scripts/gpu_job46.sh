set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_LIBS=none AB_KNOBS=chunk=DAL_GRAM_CONTIG:0,nc5=DAL_GRAM_NC:5,nc10=DAL_GRAM_NC:10,nc56=DAL_GRAM_NC:56,ant0=DAL_GRAM_ANT:0 AB_SHAPES=100000x64,200000x64,284807x30 AB_ROUNDS=7 timeout -k 10 300 python -u scripts/gram_ablate.py > gpurun_out/ab46.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ab46.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
DAL_GRAM_CONTIG=0 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_chunk.log 2>&1; rc=$?
echo "pytest chunk rc=$rc"; tail -5 gpurun_out/pytest_gpu_chunk.log
