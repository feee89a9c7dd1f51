set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/prof_shard
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/prof_shard/t -o run --output-format csv -- python3 $R/scripts/sharded_overhead.py 10 > $R/gpurun_out/prof_shard/t.log 2>&1; rc=$?; echo "t rc=$rc"
