"""Same-process A/B of the blocked K2 (dal_forest_score_blocked, density mode
with interval keys) with and without the prepared forest (ABI v10,
dal_forest_prepare: VERDICT r5 item 3).  Without it every block rebuilds the
forest's feature list, remaps its nodes and walks them by heap index (the
round-5 kernel); with it every block copies the prepared payload and walks
nodes by LDS byte address (or by heap index in a -DDAL_FOREST_BYTEA=0 build,
scripts/ab_build.sh, given with --lib: every library's prepared forest is
built by that library).  Per shape: outputs (votes, scores, both keys) must be
bit-identical across variants; then 20 back-to-back launches between two HIP
events, interleaved, median of 5 rounds.  --only prep|noprep runs one variant
of the product library (for rocprofv3 --pmc passes: instructions per node
visit = SQ_INSTS_* x 64 / (rows x trees x depth)).  Shape suffix ":normal":
N(0,1) pool.
usage: python scripts/forest_prep_ab.py [--only prep|noprep] [--lib NAME=PATH ...] [NxDxT[:normal] ...]"""
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
from dal._lib import DAL_DESCENDING, call, load  # noqa: E402
from dal.engine import PoolState, _ptr, _stream  # noqa: E402
from dal.forest import Forest  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def main():
    argv = sys.argv[1:]
    only, libs = None, {}
    while argv[:1] in (["--only"], ["--lib"]):
        if argv[0] == "--only":
            only = argv[1]
        else:
            name, path = argv[1].split("=", 1)
            libs[name] = bind(path if os.path.isabs(path) else os.path.join(REPO, path))
        argv = argv[2:]
    libs = {"cur": load(), **libs}
    shapes = argv or ["284807x30x100:normal", "2000000x256x10", "2000000x256x100", "100000x64x10"]
    dev = torch.device("cuda:0")
    for spec in shapes:
        dims, _, opt = spec.partition(":")
        n, d, T = (int(v) for v in dims.split("x"))
        dist = "normal" if opt == "normal" else "uniform"
        x = bench.upload(bench.host_pool(0, n, d, dist), dev)
        st = PoolState(x, excluded=np.arange(10), device=dev)
        dens = torch.randint(0, 1 << 40, (n,), device=dev)
        flags, _, _ = st.row_flags(torch.arange(10, n, device=dev))
        F = Forest.synthetic(T, 4, d, seed=1, dist=dist)
        inner, leaf = F.device(dev)
        used = len(np.unique(F.inner[..., 0]))
        lut = engine.device_lut("entropy", T, dev)
        s = _stream(dev)
        xb = torch.empty(int(load().dal_pool_blocked_floats(n, d)), dtype=torch.float32, device=dev)
        call("dal_pool_blocked", _ptr(x), n, d, d, _ptr(xb), s)
        nb = int(load().dal_forest_prep_bytes(d, T, 4))
        preps = {}
        for name, lib in libs.items():
            preps[name] = torch.empty(nb, dtype=torch.uint8, device=dev)
            assert lib.dal_forest_prepare(_ptr(inner), _ptr(leaf), T, 4, d, _ptr(preps[name]), nb, s) == 0
        variants = [("cur", "noprep")] if only in (None, "noprep") else []
        variants += [(name, "prep") for name in libs if only in (None, "prep")]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        outs = {v: [torch.empty(n, dtype=dt, device=dev) for dt in (torch.int32, torch.float64, torch.int64,
                                                                    torch.int64)] for v in variants}

        def run(v):
            name, mode = v
            o = outs[v]
            rc = libs[name].dal_forest_score_blocked(
                _ptr(x), _ptr(xb), _ptr(preps[name]) if mode == "prep" else 0, n, d, d, _ptr(inner), _ptr(leaf), T, 4,
                _ptr(lut), _ptr(dens), 1, 1e-6, _ptr(flags), 1.0, DAL_DESCENDING, _ptr(o[0]), _ptr(o[1]), _ptr(o[2]),
                _ptr(o[3]), s)
            assert rc == 0, rc

        for v in variants:
            run(v)
        torch.cuda.synchronize()
        same = all(all(torch.equal(a.view(torch.int64) if a.dtype == torch.float64 else a,
                                   b.view(torch.int64) if b.dtype == torch.float64 else b)
                       for a, b in zip(outs[variants[0]], outs[v])) for v in variants[1:])
        t = {v: [] for v in variants}
        for _ in range(5):
            for v in variants:
                run(v)
                e0.record()
                for _ in range(20):
                    run(v)
                e1.record()
                torch.cuda.synchronize()
                t[v].append(e0.elapsed_time(e1) / 20 * 1000)
        med = {v: statistics.median(r) for v, r in t.items()}
        base = med[variants[0]]
        line = f"{spec:24s} used {used:3d}/{d}  " + "  ".join(
            f"{v[0]}:{v[1]} {med[v]:8.2f} us ({base / med[v]:.3f}x, "
            f"{n * (4 * used + 37) / med[v] / 1e3:.0f} GB/s)" for v in variants)
        print(line + f"  bits identical: {same}", flush=True)
        del x, st, xb, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
