set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/pmc58
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --warm-steps 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc58/f -o run --output-format csv -- $B > $R/gpurun_out/pmc58/f.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc58/w -o run --output-format csv -- $B > $R/gpurun_out/pmc58/w.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R && for k in gram_sym2 forest_score normalize_split canon_colsum_partials; do echo "== $k"; python3 scripts/pmc_summary.py gpurun_out/pmc58 $k; done
