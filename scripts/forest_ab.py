"""A/B: dal_forest_score lanes-per-row (DAL_FOREST_TPR) on the BASELINE
shapes, HIP events on the launch stream, same process.
usage: python scripts/forest_ab.py [reps] [NxDxT | sweepT]"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np
import torch
from dal import engine
from dal._lib import DAL_DESCENDING
from dal.forest import Forest
import bench

dev = torch.device("cuda:0")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
only = sys.argv[2] if len(sys.argv) > 2 else None  # e.g. "284807x30": one shape


def timed(state, forest, lut, flags, dens, err):
    state.forest_events = []
    for _ in range(reps):
        out = engine.forest_score(state, forest, lut, flags, DAL_DESCENDING, density=dens,
                                  density_err=err, want_hi=True)
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in state.forest_events[5:]]
    state.forest_events = None
    return float(np.median(ms)), out


SHAPES = ((284807, 30, 100, "normal"), (100000, 64, 10, "uniform"),
                      (100000, 64, 100, "uniform"), (2000000, 256, 10, "uniform"), (2000000, 256, 100, "uniform"),
                      (2000000, 32, 100, "uniform"))
if only and only.startswith("sweepT"):  # fixed cost vs trees at the config-3 shape
    SHAPES = tuple((284807, 30, t, "normal") for t in (1, 4, 16, 50, 100))
    only = None
for n, d, t, dist in SHAPES:
    if only and only != f"{n}x{d}x{t}":
        continue
    x = bench.upload(bench.host_pool(0, n, d, dist), dev)
    forest = Forest.synthetic(t, 4, d, seed=1, dist=dist)
    st = engine.PoolState(x, excluded=np.arange(10), device=dev)
    flags, _, _ = st.row_flags(torch.arange(10, n, device=dev))
    lut = engine.device_lut("entropy", t, dev)
    dens = torch.zeros(st.n_pad, dtype=torch.int64, device=dev)
    err = 1e-3
    res = {}
    knob = os.environ.get("AB_KNOB", "DAL_FOREST_TPR")
    vals = os.environ.get("AB_VALS", "1,2,4").split(",")
    variants = (("default", None),) + tuple((f"{knob}={v}", v) for v in vals)
    for name, val in variants:
        if val is None:
            os.environ.pop(knob, None)
        else:
            os.environ[knob] = val
        res[name] = timed(st, forest, lut, flags, dens, err)
    os.environ.pop(knob, None)
    # scores hold NaN for excluded rows: compare bit patterns
    bits = lambda o: [a.view(torch.int64) if a.dtype == torch.float64 else a for a in o]
    ref = bits(res["default"][1])
    row_bytes = d * 4 + 1 + 8 + 4 + 8 + 16
    for name, _ in variants:
        ms, out = res[name]
        same = all(torch.equal(a, b) for a, b in zip(ref, bits(out)))
        print(f"n={n} d={d} T={t} kernel={name}: {ms * 1e3:.1f} us "
              f"({n * row_bytes / ms / 1e6:.0f} GB/s algorithmic) identical={same}", flush=True)
