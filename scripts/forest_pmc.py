"""dal_forest_score at one BASELINE shape, a few launches, for rocprofv3 --pmc
(FETCH_SIZE / WRITE_SIZE in separate passes).  usage: python scripts/forest_pmc.py NxDxT[:blocked] [reps] [LIB.so]
(:blocked: dal_forest_score_blocked over the pool's blocked copy, built first;
LIB.so: an A/B build, scripts/ab_build.sh, instead of the product library)"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dal import _lib, engine  # noqa: E402

if len(sys.argv) > 3:  # bind an A/B build in place of the product library
    import ctypes

    lib = ctypes.CDLL(os.path.abspath(sys.argv[3]))
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib._lib = lib
from dal._lib import DAL_DESCENDING  # noqa: E402
from dal.forest import Forest  # noqa: E402

dev = torch.device("cuda:0")
shape, _, mode = sys.argv[1].partition(":")
n, d, t = (int(v) for v in shape.split("x"))
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dist = "normal" if d == 30 else "uniform"
x = bench.upload(bench.host_pool(0, n, d, dist), dev)
forest = Forest.synthetic(t, 4, d, seed=1, dist=dist)
st = engine.PoolState(x, excluded=np.arange(10), device=dev)
flags, _, _ = st.row_flags(torch.arange(10, n, device=dev))
lut = engine.device_lut("entropy", t, dev)
dens = torch.zeros(st.n_pad, dtype=torch.int64, device=dev)
xb = st.blocked_pool(forest) if mode == "blocked" else None
if mode == "blocked" and xb is None:
    raise SystemExit("the blocked path does not apply to this shape")
for _ in range(reps):
    engine.forest_score(st, forest, lut, flags, DAL_DESCENDING, density=dens, density_err=1e-3, want_hi=True, xb=xb)
torch.cuda.synchronize()
print("ok", n, d, t, reps, mode or "row-major")
