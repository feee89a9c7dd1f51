set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o prof --output-format csv -- python3 bench.py --config 3 --steps 3 --warmup 1 --warm-steps 10 --no-cpu-baseline > gpurun_out/prof3.log 2>&1; rc=$?
echo "rc=$rc"
