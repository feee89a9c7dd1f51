set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-3000
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1; rc=$?; echo "bench c3 rc=$rc"; tail -1 gpurun_out/bench_c3.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/pmc_sym
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_c2.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --warm-steps 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_sym/f -o run --output-format csv -- $B > $R/gpurun_out/pmc_sym/f.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_sym/w -o run --output-format csv -- $B > $R/gpurun_out/pmc_sym/w.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
export AB_KINDS=sym AB_SHAPES=100000x64
P="python3 $R/scripts/gram_split_ab.py 1"
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d $R/gpurun_out/pmc_sym/p1 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sym/p1.log 2>&1; rc=$?; echo "p1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_LDS_DATA_FIFO_FULL -d $R/gpurun_out/pmc_sym/p2 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sym/p2.log 2>&1; rc=$?; echo "p2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_sym/p3 -o run --output-format csv -- $P > $R/gpurun_out/pmc_sym/p3.log 2>&1; rc=$?; echo "p3 rc=$rc"
cd $R && python3 scripts/pmc_summary.py gpurun_out/pmc_sym gram_sym_kernel
