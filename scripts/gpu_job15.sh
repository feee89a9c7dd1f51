set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_KINDS=split0,split timeout -k 10 240 python -u scripts/gram_split_ab.py 3 > gpurun_out/split_ab2.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/split_ab2.log
[ $rc -eq 0 ] || exit $rc
mkdir -p $R/gpurun_out/pmc_sp2
cd /tmp && export TMPDIR=/tmp
export AB_KINDS=split AB_SHAPES=100000x64
P="python3 $R/scripts/gram_split_ab.py 1"
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d $R/gpurun_out/pmc_sp2/p1 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sp2/p1.log 2>&1; rc=$?; echo "p1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_sp2/p4 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sp2/p4.log 2>&1; rc=$?; echo "p4 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_sp2/p3 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sp2/p3.log 2>&1; rc=$?; echo "p3 rc=$rc"
cd $R && python3 scripts/pmc_summary.py gpurun_out/pmc_sp2 gram_split_kernel
