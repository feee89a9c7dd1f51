#!/bin/bash
# One parameterised GPU-box runner (replaces the round-1 one-shot job files).
#
#   gpurun --timeout 900 -- bash scripts/gpu_run.sh STEP [STEP ...]
#
# STEP (run in order, each under its own time limit; the first failure ends
# the call -- no GPU step runs after a fault, abort or timeout):
#   tests[=EXPR]          pytest -m gpu (optionally -k EXPR, ',' = space) -> gpurun_out/pytest_gpu.log
#   smoke                 __graft_entry__.smoke()             -> gpurun_out/smoke.log
#   bench[=ARGS]          python bench.py ARGS (',' = space)  -> gpurun_out/bench_<n>.log
#                         (full result: gpurun_out/bench_full_<n>.json)
#   sharded[=ARGS]        DAL_BENCH_SHARDED=1 python bench.py ARGS: --gpus 1 through dal/parallel.py on a
#                         one-rank RCCL group -> gpurun_out/sharded_<n>.log
#   gloo=N[=ARGS]         bench.py on N gloo ranks sharing the one GPU (torch.distributed.run)
#                         -> gpurun_out/gloo_<n>.log
#   selfgloo=N[=ARGS]     bench.py --gpus N on gloo with NO outside launcher (bench.py starts its ranks)
#                         -> gpurun_out/selfgloo_<n>.log
#   stats=TAG[=ARGS]      rocprofv3 --kernel-trace --stats of bench.py ARGS -> gpurun_out/prof_TAG/
#   pmc=TAG=CTRS[=ARGS]   rocprofv3 --pmc CTRS (',' = space) of bench.py ARGS -> gpurun_out/pmc_TAG/
#   pmcpy=TAG=CTRS=SCRIPT[=ARGS]  rocprofv3 --pmc CTRS of python SCRIPT ARGS -> gpurun_out/pmc_TAG/
#   py=SCRIPT[=ARGS]      python SCRIPT ARGS                  -> gpurun_out/py_<n>.log
#   trace=TAG=SCRIPT[=ARGS]  rocprofv3 --kernel-trace of python SCRIPT ARGS -> gpurun_out/trace_TAG/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%=*}
  rest=""
  [[ "$step" == *=* ]] && rest=${step#*=}
  case "$kind" in
    tests)
      k=()
      [ -n "$rest" ] && k=(-k "${rest//,/ }")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${k[@]}" \
        > gpurun_out/pytest_gpu.log 2>&1
      rc=$?
      echo "[$n] tests rc=$rc: $(tail -1 gpurun_out/pytest_gpu.log)"
      ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?
      echo "[$n] smoke rc=$rc: $(tail -1 gpurun_out/smoke.log)"
      ;;
    bench)
      timeout -k 10 900 python -u bench.py ${rest//,/ } --out gpurun_out/bench_full_$n.json \
        > gpurun_out/bench_$n.log 2>&1
      rc=$?
      echo "[$n] bench ${rest//,/ } rc=$rc"
      tail -1 gpurun_out/bench_$n.log | cut -c1-600
      ;;
    sharded)
      DAL_BENCH_SHARDED=1 timeout -k 10 900 python -u bench.py ${rest//,/ } --out gpurun_out/sharded_full_$n.json \
        > gpurun_out/sharded_$n.log 2>&1
      rc=$?
      echo "[$n] sharded ${rest//,/ } rc=$rc"
      tail -1 gpurun_out/sharded_$n.log | cut -c1-600
      ;;
    gloo)
      np=${rest%%=*}
      args=""
      [[ "$rest" == *=* ]] && args=${rest#*=}
      DAL_BENCH_BACKEND=gloo timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $np --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $np \
        ${args//,/ } --out gpurun_out/gloo_full_$n.json > gpurun_out/gloo_$n.log 2>&1
      rc=$?
      echo "[$n] gloo $np ${args//,/ } rc=$rc"
      tail -1 gpurun_out/gloo_$n.log | cut -c1-600
      ;;
    selfgloo)
      np=${rest%%=*}
      args=""
      [[ "$rest" == *=* ]] && args=${rest#*=}
      env -u WORLD_SIZE DAL_BENCH_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus $np \
        ${args//,/ } --out gpurun_out/selfgloo_full_$n.json > gpurun_out/selfgloo_$n.log 2>&1
      rc=$?
      echo "[$n] selfgloo $np ${args//,/ } rc=$rc"
      tail -1 gpurun_out/selfgloo_$n.log | cut -c1-600
      ;;
    stats)
      tag=${rest%%=*}
      args=""
      [[ "$rest" == *=* ]] && args=${rest#*=}
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
        python3 -u bench.py ${args//,/ } > gpurun_out/prof_$tag.log 2>&1
      rc=$?
      echo "[$n] stats $tag rc=$rc"
      tail -1 gpurun_out/prof_$tag.log | cut -c1-300
      ;;
    pmc)
      tag=${rest%%=*}
      r2=${rest#*=}
      ctrs=${r2%%=*}
      args=""
      [[ "$r2" == *=* ]] && args=${r2#*=}
      timeout -s KILL 240 rocprofv3 --pmc ${ctrs//,/ } --output-format csv -d gpurun_out/pmc_$tag -o run -- \
        python3 -u bench.py ${args//,/ } > gpurun_out/pmc_$tag.log 2>&1
      rc=$?
      echo "[$n] pmc $tag rc=$rc"
      ;;
    pmcpy)
      tag=${rest%%=*}
      r2=${rest#*=}
      ctrs=${r2%%=*}
      r3=${r2#*=}
      scr=${r3%%=*}
      args=""
      [[ "$r3" == *=* ]] && args=${r3#*=}
      timeout -s KILL 240 rocprofv3 --pmc ${ctrs//,/ } --output-format csv -d gpurun_out/pmc_$tag -o run -- \
        python3 -u $scr ${args//,/ } > gpurun_out/pmc_$tag.log 2>&1
      rc=$?
      echo "[$n] pmcpy $tag rc=$rc"
      ;;
    trace)
      tag=${rest%%=*}
      r2=${rest#*=}
      scr=${r2%%=*}
      args=""
      [[ "$r2" == *=* ]] && args=${r2#*=}
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$tag -o run -- \
        python3 -u $scr ${args//,/ } > gpurun_out/trace_$tag.log 2>&1
      rc=$?
      echo "[$n] trace $tag rc=$rc"
      ;;
    py)
      scr=${rest%%=*}
      args=""
      [[ "$rest" == *=* ]] && args=${rest#*=}
      timeout -k 10 900 python -u $scr ${args//,/ } > gpurun_out/py_$n.log 2>&1
      rc=$?
      echo "[$n] py $scr rc=$rc"
      tail -5 gpurun_out/py_$n.log | cut -c1-600
      ;;
    *)
      echo "unknown step $step"
      exit 2
      ;;
  esac
  [ $rc -eq 0 ] || exit $rc
done
