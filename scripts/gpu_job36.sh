set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/pmc_sym2
cd /tmp && export TMPDIR=/tmp
export AB_KINDS=sym AB_SHAPES=100000x64
P="python3 $R/scripts/gram_split_ab.py 1"
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $R/gpurun_out/pmc_sym2/p1 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sym2/p1.log 2>&1; rc=$?; echo "p1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD -d $R/gpurun_out/pmc_sym2/p2 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sym2/p2.log 2>&1; rc=$?; echo "p2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_sym2/p3 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sym2/p3.log 2>&1; rc=$?; echo "p3 rc=$rc"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc_sym2/t -o run --output-format csv -- $P > $R/gpurun_out/pmc_sym2/t.log 2>&1; rc=$?; echo "t rc=$rc"
cd $R && python3 scripts/pmc_summary.py gpurun_out/pmc_sym2 gram_sym2
grep -h gram_sym2 gpurun_out/pmc_sym2/t/run_kernel_stats.csv | cut -c1-200
