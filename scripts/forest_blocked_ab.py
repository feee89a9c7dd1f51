"""Same-process A/B of K2 (dal_forest_score, density mode with interval keys):
the row-major tile (dal_forest_score) against the blocked feature-major path
(dal_pool_blocked once, then dal_forest_score_blocked, which reads only the
features the forest tests).  Per shape: outputs (votes, scores, both keys)
must be bit-identical; then 20 back-to-back launches between two HIP events,
interleaved row/blocked, median of 5 rounds.  Shape suffixes: ":us"
uncertainty mode (no density), ":normal" N(0,1) pool.
usage: python scripts/forest_blocked_ab.py [NxDxT[:us|:normal] ...]"""
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

if os.environ.get("DAL_AB_LIB"):  # an A/B build in place of the product library
    import ctypes

    _ab = ctypes.CDLL(os.path.abspath(os.environ["DAL_AB_LIB"]))
    for _name, (_res, _args) in _lib.SIGNATURES.items():
        getattr(_ab, _name).restype = _res
        getattr(_ab, _name).argtypes = _args
    _lib._lib = _ab
from dal._lib import DAL_DESCENDING, call, load  # noqa: E402
from dal.engine import PoolState, _ptr, _stream  # noqa: E402
from dal.forest import Forest  # noqa: E402


def main():
    shapes = sys.argv[1:] or ["2000000x256x10", "1999963x256x10", "2000000x256x10:us", "100000x256x10",
                              "500000x512x10", "2000000x256x8:normal"]
    dev = torch.device("cuda:0")
    for spec in shapes:
        dims, _, opt = spec.partition(":")
        n, d, T = (int(v) for v in dims.split("x"))
        dist = "normal" if opt == "normal" else "uniform"
        x = bench.upload(bench.host_pool(0, n, d, dist), dev)
        st = PoolState(x, excluded=np.arange(10), device=dev)
        dens = None if opt == "us" else torch.randint(0, 1 << 40, (n,), device=dev)
        flags, _, _ = st.row_flags(torch.arange(10, n, device=dev))
        F = Forest.synthetic(T, 4, d, seed=1, dist=dist)
        inner, leaf = F.device(dev)
        used = len(np.unique(F.inner[..., 0]))
        lut = engine.device_lut("entropy", T, dev)
        s = _stream(dev)
        xb = torch.empty(int(load().dal_pool_blocked_floats(n, d)), dtype=torch.float32, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call("dal_pool_blocked", _ptr(x), n, d, d, _ptr(xb), s)
        e1.record()
        torch.cuda.synchronize()
        t_blk = e0.elapsed_time(e1) * 1000
        outs = {m: [torch.empty(n, dtype=dt, device=dev) for dt in (torch.int32, torch.float64, torch.int64,
                                                                    torch.int64)] for m in ("row", "blocked")}
        dptr, dkind = (None, 0) if dens is None else (_ptr(dens), 1)

        def run(m):
            o = outs[m]
            tail = (_ptr(inner), _ptr(leaf), T, 4, _ptr(lut), dptr, dkind, 1e-6, _ptr(flags), 1.0, DAL_DESCENDING,
                    _ptr(o[0]), _ptr(o[1]), _ptr(o[2]), _ptr(o[3]), s)
            if m == "row":
                call("dal_forest_score", _ptr(x), n, d, d, *tail)
            else:
                call("dal_forest_score_blocked", _ptr(x), _ptr(xb), 0, n, d, d, *tail)

        for m in outs:
            run(m)
        torch.cuda.synchronize()
        same = all(torch.equal(a.view(torch.int64) if a.dtype == torch.float64 else a,
                               b.view(torch.int64) if b.dtype == torch.float64 else b)
                   for a, b in zip(outs["row"], outs["blocked"]))
        t = {m: [] for m in outs}
        for _ in range(5):
            for m in outs:
                run(m)
                e0.record()
                for _ in range(20):
                    run(m)
                e1.record()
                torch.cuda.synchronize()
                t[m].append(e0.elapsed_time(e1) / 20 * 1000)
        tr, tb = statistics.median(t["row"]), statistics.median(t["blocked"])
        gb_row = n * (4 * d + 37) / tb / 1e3
        gb_used = n * (4 * used + 37) / tb / 1e3
        print(f"{spec:22s} used {used:3d}/{d}  row {tr:8.1f} us  blocked {tb:8.1f} us ({tr / tb:.2f}x; "
              f"{gb_used:.0f} GB/s of used-feature bytes, {gb_row:.0f} GB/s row-equivalent)  "
              f"copy {t_blk:.0f} us  bits identical: {same}", flush=True)
        del x, st, xb, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
