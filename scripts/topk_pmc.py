"""K3 (dal_dw_select) at one BASELINE shape, a few eager calls, for
rocprofv3 --pmc (FETCH_SIZE / WRITE_SIZE in separate passes) and
--kernel-trace: the pool's density is computed first (Gram), then the
forest scores, then `reps` dal_dw_select calls.  The per-call traffic is the
sum over the kernels between two calls' first radix launches.
usage: python scripts/topk_pmc.py NxD [reps] [trees]  (d = 30: config 3's N(0,1) pool)"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dal import engine  # noqa: E402
from dal._lib import DAL_DESCENDING  # noqa: E402
from dal.forest import Forest  # noqa: E402

dev = torch.device("cuda:0")
n, d = (int(v) for v in sys.argv[1].split("x"))
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
trees = int(sys.argv[3]) if len(sys.argv) > 3 else 10
x = bench.upload(bench.host_pool(0, n, d, "normal" if d == 30 else "uniform"), dev)
forest = Forest.synthetic(trees, 4, d, seed=1)
st = engine.PoolState(x, excluded=np.arange(10), device=dev)
dens = st.density_fixed()
flags, _, _ = st.row_flags(torch.arange(10, n, device=dev))
lut = engine.device_lut("entropy", trees, dev)
votes, scores, klo, khi = engine.forest_score(st, forest, lut, flags, DAL_DESCENDING, density=dens,
                                              density_err=engine.density_error(st), want_hi=True)
cs = st.colsum()
torch.cuda.synchronize()
for _ in range(reps):
    idx, sc, _ = engine.dw_select_local(st, flags, votes, klo, khi, lut, 100, 1.0, cs)
torch.cuda.synchronize()
print("ok", n, d, reps, idx[:4].tolist())
