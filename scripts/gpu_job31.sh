set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_LIBS=none AB_KNOBS=nc4=DAL_GRAM_NC:4,nc7=DAL_GRAM_NC:7,nc10=DAL_GRAM_NC:10,nc14=DAL_GRAM_NC:14,nc20=DAL_GRAM_NC:20,nc49=DAL_GRAM_NC:49 timeout -k 10 200 python -u scripts/gram_ablate.py > gpurun_out/ablate4.log 2>&1; rc=$?
echo "ablate rc=$rc"; grep -v amdgpu.ids gpurun_out/ablate4.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; python3 -c "
import json
d=json.loads(open('gpurun_out/bench_default.log').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
