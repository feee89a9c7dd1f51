set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_VARIANTS=nw4,nw8 timeout -k 10 300 python -u scripts/maxcos_ab.py 5 > gpurun_out/maxcos_ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/maxcos_ab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_maxcos.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?; echo "c5 rc=$rc"; python3 -c "
import json
d=json.loads(open('gpurun_out/bench_c5.log').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['value'])"
mkdir -p gpurun_out/prof_c5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5/trace -o run --output-format csv -- python3 $R/bench.py --config 5 --steps 3 --warmup 1 > $R/gpurun_out/prof_c5/trace.log 2>&1; echo "prof rc=$?"
