"""Per-block timeline of the blocked K2 (dal_forest_score_blocked) from a
timing-only build (scripts/variant_build.py with a patch stamping
s_memrealtime at each block's start and end into a device array read back
by dal_ft_trace): the span of the launch, the blocks' start offsets and
durations, and how many blocks are alive over time.
usage: DAL_AB_LIB=ab/fttrace/libdal.so python scripts/k2_block_timeline.py NxDxT [reps]"""
import ctypes
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dal import _lib, engine  # noqa: E402

lib = ctypes.CDLL(os.path.abspath(os.environ["DAL_AB_LIB"]))
for name, (res, args) in _lib.SIGNATURES.items():
    if hasattr(lib, name):
        getattr(lib, name).restype = res
        getattr(lib, name).argtypes = args
_lib._lib = lib
from dal._lib import DAL_DESCENDING  # noqa: E402
from dal.forest import Forest  # noqa: E402

TICK_NS = 10.0  # s_memrealtime: 100 MHz

dev = torch.device("cuda:0")
n, d, t = (int(v) for v in sys.argv[1].split("x"))
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dist = "normal" if d == 30 else "uniform"
x = bench.upload(bench.host_pool(0, n, d, dist), dev)
forest = Forest.synthetic(t, 4, d, seed=1, dist=dist)
st = engine.PoolState(x, excluded=np.arange(10), device=dev)
flags, _, _ = st.row_flags(torch.arange(10, n, device=dev))
lut = engine.device_lut("entropy", t, dev)
dens = torch.zeros(st.n_pad, dtype=torch.int64, device=dev)
xb = st.blocked_pool(forest)
for _ in range(reps):
    engine.forest_score(st, forest, lut, flags, DAL_DESCENDING, density=dens, density_err=1e-3, want_hi=True, xb=xb)
torch.cuda.synchronize()
buf = np.zeros((4, 16384), dtype=np.uint64)
assert lib.dal_ft_trace(ctypes.c_void_p(buf.ctypes.data)) == 0
grid = int(buf[3, 0])
tiles = (n + 63) // 64
s, e = buf[0, :grid].astype(np.int64), buf[2, :grid].astype(np.int64)
t0 = s.min()
span = (e.max() - t0) * TICK_NS / 1e3
dur = (e - s) * TICK_NS / 1e3
off = (s - t0) * TICK_NS / 1e3
per = np.array([len(range(b, tiles, grid)) for b in range(grid)])
print(f"{n}x{d}x{t}: grid {grid} blocks, {tiles} tiles ({tiles / grid:.2f} per block), span {span:.1f} us")
print(f"  start offset us: median {np.median(off):.2f}  p90 {np.percentile(off, 90):.2f}  max {off.max():.2f}")
for k in sorted(set(per.tolist())):
    m = per == k
    print(f"  blocks with {k} tiles: {m.sum():5d}  duration us median {np.median(dur[m]):.2f}  "
          f"p10 {np.percentile(dur[m], 10):.2f}  p90 {np.percentile(dur[m], 90):.2f}  max {dur[m].max():.2f}")
print(f"  block-time / (grid x span): {dur.sum() / (grid * span):.3f}")
bins = np.arange(0.0, span + 1.0, max(span / 20, 0.5))
alive = [int(((off <= b) & (off + dur > b)).sum()) for b in bins]
print("  blocks alive at t (us): " + "  ".join(f"{b:.1f}:{a}" for b, a in zip(bins, alive)))
