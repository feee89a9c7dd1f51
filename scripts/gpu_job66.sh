set -u
cd $GRAFT_REPO_ROOT
run() {
  env "$@" timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline --warm-steps 0 > gpurun_out/g3.log 2>&1; rc=$?
  echo "$* rc=$rc $(tail -1 gpurun_out/g3.log | grep -o '"launch_ms": [0-9.]*' | head -1) $(tail -1 gpurun_out/g3.log | grep -o '"frac": [0-9.]*' | head -1)"
  return $rc
}
run X=0 && run DAL_GRAM_CONTIG=1 && run DAL_GRAM_CONTIG=0 && run DAL_GRAM_SYM=1 && run X=0 && run DAL_GRAM_CONTIG=1
