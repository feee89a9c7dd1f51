set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | head -20 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
export AB_KINDS=sym,symk1 AB_SHAPES=100000x64,200000x30,500000x256
timeout -k 10 240 python -u scripts/gram_split_ab.py 3 > gpurun_out/sg_ab4.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/sg_ab4.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; python3 -c "
import json
d=json.loads(open('gpurun_out/bench_default.log').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['value'])"
DAL_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 3 --warmup 1 > gpurun_out/bench_gloo4.log 2>&1; rc=$?; echo "gloo4 rc=$rc"; grep metric gpurun_out/bench_gloo4.log | cut -c1-200
