set -u
R=$GRAFT_REPO_ROOT
cd $R
AB_KINDS=split16,sym timeout -k 10 240 python -u scripts/gram_split_ab.py 3 > gpurun_out/split_ab4.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/split_ab4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|error" gpurun_out/pytest_gpu.log | head -30 | cut -c1-300
