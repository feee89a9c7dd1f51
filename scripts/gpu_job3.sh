set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 480 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log | cut -c1-300
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/gram_ab.py 3 > gpurun_out/gram_ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/gram_ab.log | grep n=
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d $R/gpurun_out/pmc_sq -o run --output-format csv -- python3 $R/scripts/gram_ab.py 1 > $R/gpurun_out/pmc_sq.log 2>&1; rc=$?; echo "pmc rc=$rc"
