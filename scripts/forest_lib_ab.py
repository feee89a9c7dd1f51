"""Same-process A/B of dal_forest_score (K2, density mode with interval keys)
between two builds of libdal.so: ab/libdal_base.so (the committed kernel) and
the current in-tree library.  Per shape: both libraries' outputs (votes,
scores, both keys) must be bit-identical; then 20 back-to-back launches
between two HIP events, interleaved A/B/A/B, median of the rounds.
usage: python scripts/forest_lib_ab.py [NxDxT[:normal] ...]   (AB_BASE / AB_NEW: other library paths)"""
import ctypes
import os
import statistics
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dal import _lib, engine  # noqa: E402
from dal._lib import DAL_DESCENDING  # noqa: E402
from dal.engine import PoolState, _ptr, _stream  # noqa: E402
from dal.forest import Forest  # noqa: E402

c_i64, c_p, c_int, c_dbl = ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_double


def bind(path):
    lib = ctypes.CDLL(path)
    f = lib.dal_forest_score
    f.argtypes = [c_p, c_i64, c_i64, c_i64, c_p, c_p, ctypes.c_int32, ctypes.c_int32, c_p, c_p, c_int, c_dbl, c_p,
                  c_dbl, c_int, c_p, c_p, c_p, c_p, c_p]
    return lib


def main():
    shapes = [a for a in sys.argv[1:]] or ["100000x64x10", "284807x30x100:normal", "2000000x256x10",
                                           "2000000x32x100", "2000000x256x100"]
    dev = torch.device("cuda:0")
    base = os.environ.get("AB_BASE", os.path.join(REPO, "ab", "libdal_base.so"))
    libs = {"base": bind(base), "new": bind(os.environ.get("AB_NEW", _lib.LIB_PATH))}
    for spec in shapes:
        dims, _, dist = spec.partition(":")
        n, d, T = (int(v) for v in dims.split("x"))
        x = bench.upload(bench.host_pool(0, n, d, dist or "uniform"), dev)
        st = PoolState(x, excluded=np.arange(10), device=dev)
        dens = st.density_fixed() if n * d <= 64_000_000 else torch.randint(0, 1 << 40, (n,), device=dev)
        flags, _, _ = st.row_flags(torch.arange(10, n, device=dev))
        F = Forest.synthetic(T, 4, d, seed=1, dist=dist or "uniform")
        inner, leaf = F.device(dev)
        lut = engine.device_lut("entropy", T, dev)
        outs = {}
        for name, lib in libs.items():
            o = [torch.empty(n, dtype=dt, device=dev) for dt in (torch.int32, torch.float64, torch.int64, torch.int64)]
            outs[name] = o
        s = _stream(dev)

        def run(name):
            o = outs[name]
            rc = libs[name].dal_forest_score(_ptr(x), n, d, d, _ptr(inner), _ptr(leaf), T, 4, _ptr(lut), _ptr(dens),
                                             1, 1e-6, _ptr(flags), 1.0, DAL_DESCENDING, _ptr(o[0]), _ptr(o[1]),
                                             _ptr(o[2]), _ptr(o[3]), s)
            assert rc == 0, rc

        for name in libs:
            run(name)
        torch.cuda.synchronize()
        same = all(torch.equal(a.view(torch.int64) if a.dtype == torch.float64 else a,
                               b.view(torch.int64) if b.dtype == torch.float64 else b)
                   for a, b in zip(outs["base"], outs["new"]))
        t = {name: [] for name in libs}
        for _ in range(5):
            for name in libs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                run(name)
                e0.record()
                for _ in range(20):
                    run(name)
                e1.record()
                torch.cuda.synchronize()
                t[name].append(e0.elapsed_time(e1) / 20 * 1000)
        print(f"{spec:24s} base {statistics.median(t['base']):8.1f} us  new {statistics.median(t['new']):8.1f} us"
              f"  bits identical: {same}", flush=True)


if __name__ == "__main__":
    main()
