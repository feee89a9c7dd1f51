set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/colsum_stream_ab.py 2>&1 | grep -v amdgpu.ids
