set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_KINDS=split32,split16 timeout -k 10 240 python -u scripts/gram_split_ab.py 3 > gpurun_out/split_ab3.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/split_ab3.log
[ $rc -eq 0 ] || exit $rc
mkdir -p $R/gpurun_out/pmc_sp3
cd /tmp && export TMPDIR=/tmp
export AB_KINDS=split16 AB_SHAPES=100000x64
P="python3 $R/scripts/gram_split_ab.py 1"
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d $R/gpurun_out/pmc_sp3/p1 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sp3/p1.log 2>&1; rc=$?; echo "p1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_DATA_FIFO_FULL -d $R/gpurun_out/pmc_sp3/p2 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sp3/p2.log 2>&1; rc=$?; echo "p2 rc=$rc"
cd $R && python3 scripts/pmc_summary.py gpurun_out/pmc_sp3 gram_split_kernel
