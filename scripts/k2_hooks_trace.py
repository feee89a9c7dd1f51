"""K2 (forest_score_kernel) with and without the warm step's hooks, same
process, for rocprofv3 --kernel-trace: (a) eager dal_forest_score with the
cached density (no hooks), (b) the warm density step (dal_dw_step through the
plan: mark stamps -> row flags, group-minimum fold), alternated.
usage: python scripts/k2_hooks_trace.py [CONFIG]"""
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

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "4"]
n, d, trees, dist = cfg["n"], cfg["d"], cfg["trees"], cfg["dist"]
dev = torch.device("cuda:0")
x = bench.upload(bench.host_pool(0, n, d, dist), dev)
forest = Forest.synthetic(trees, 4, d, seed=1, dist=dist)
unl = torch.arange(10, n, device=dev, dtype=torch.int64)
st = engine.PoolState(x, excluded=np.arange(10), device=dev)
engine.density_step(st, unl, forest, 100)  # cold: density cached
dens = st.density_fixed()
flags, _, _ = st.row_flags(unl)
lut = engine.device_lut("entropy", trees, dev)
for _ in range(5):
    engine.forest_score(st, forest, lut, flags, DAL_DESCENDING, density=dens,
                        density_err=engine.density_error(st), want_hi=True)
    torch.cuda.synchronize()
    engine.density_step(st, unl, forest, 100)
    torch.cuda.synchronize()
print("ok")
