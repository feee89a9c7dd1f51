set -u
R=$GRAFT_REPO_ROOT
cd $R
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/tl -o tl --output-format csv -- python3 scripts/step_timeline.py > gpurun_out/tl.log 2>&1; rc=$?
echo "prof rc=$rc"; tail -2 gpurun_out/tl.log
[ $rc -eq 0 ] || exit $rc
python3 scripts/step_timeline.py --analyse gpurun_out/tl > gpurun_out/tl_summary.txt; cat gpurun_out/tl_summary.txt
