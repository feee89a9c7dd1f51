set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_sp
cd /tmp && export TMPDIR=/tmp
export AB_KINDS=split AB_SHAPES=100000x64
P="python3 $R/scripts/gram_split_ab.py 1"
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d $R/gpurun_out/pmc_sp/p1 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sp/p1.log 2>&1; rc=$?; echo "p1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_DATA_FIFO_FULL -d $R/gpurun_out/pmc_sp/p2 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sp/p2.log 2>&1; rc=$?; echo "p2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_sp/p3 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sp/p3.log 2>&1; rc=$?; echo "p3 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_sp/p4 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sp/p4.log 2>&1; rc=$?; echo "p4 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_sp/p5 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sp/p5.log 2>&1; rc=$?; echo "p5 rc=$rc"
cd $R && python3 scripts/pmc_summary.py gpurun_out/pmc_sp gram_split_kernel
