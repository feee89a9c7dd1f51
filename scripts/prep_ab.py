"""Same-process A/B of the Gram's O(N*D) side launches across builds of
libdal.so (scripts/ab_build.sh): the fused prep (dal_prep_split: row norms,
the two-term fp16 split, the canonical column-sum partials), the
compensation's closed-form remainder (dal_gram_sym_residual: sigma, scan,
per-row dots) and the column-sum reduce.  Every output is compared bit for
bit against the first build, then each call is timed on its own with HIP
events, interleaved over the builds (median over the rounds).

usage: python scripts/prep_ab.py NAME=PATH [NAME=PATH ...] -- [NxD ...]
       (d = 30: config 3's N(0,1) pool; first NAME is the reference)"""
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
from dal import _lib  # noqa: E402
from dal._lib import DAL_CANON_CHUNK  # noqa: E402
from dal.engine import PoolState, _ptr, _stream  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
    return lib


def chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} returned {rc}")


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    specs = [a.split("=", 1) for a in argv[:cut]]
    shapes = argv[cut + 1:] or ["100000x64", "284807x30", "2000000x256"]
    libs = {name: bind(os.path.join(REPO, path) if not os.path.isabs(path) else path) for name, path in specs}
    names = list(libs)
    rounds = int(os.environ.get("AB_ROUNDS", "7"))
    dev = torch.device("cuda:0")
    s = _stream(dev)
    for sh in shapes:
        n, d = (int(v) for v in sh.split("x"))
        _lib._lib = libs[names[0]]
        x = bench.upload(bench.host_pool(0, n, d, "normal" if d == 30 else "uniform"), dev)
        st = PoolState(x, excluded=np.arange(10), device=dev)
        n_pad, d_pad = st.n_pad, st.d_pad
        nb = st.nb_active()
        nrb = n_pad // 256
        chunks = (n + DAL_CANON_CHUNK - 1) // DAL_CANON_CHUNK
        wsb = int(libs[names[0]].dal_gram_sym_residual_workspace_bytes(nb, nrb, d_pad))
        ws = torch.empty(wsb + 256, dtype=torch.uint8, device=dev)
        wsp = (_ptr(ws) + 255) // 256 * 256
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        out = {}

        def bufs(name):
            if name not in out:
                out[name] = dict(
                    ops=torch.empty((n_pad, 2 * d_pad), dtype=torch.int16, device=dev),
                    norm=torch.empty(n, dtype=torch.float64, device=dev),
                    parts=torch.empty((chunks, d), dtype=torch.float64, device=dev),
                    acc=torch.empty(n_pad, dtype=torch.int64, device=dev),
                    res=torch.zeros(nb * 256, dtype=torch.int64, device=dev),
                    cs=torch.empty(d, dtype=torch.float64, device=dev))
            return out[name]

        def prep(name):
            b, lib = bufs(name), libs[name]
            chk(lib.dal_prep_split(_ptr(x), n, d, d, _ptr(st.flags), n_pad, d_pad, _ptr(b["ops"]),
                                   _ptr(b["norm"]), _ptr(b["parts"]), _ptr(b["acc"]), _ptr(status), s),
                "dal_prep_split")

        def resid(name):
            b, lib = bufs(name), libs[name]
            chk(lib.dal_gram_sym_residual(_ptr(b["ops"]), nb, 0, nrb, d_pad, _ptr(b["res"]), wsp, wsb, s),
                "dal_gram_sym_residual")

        def reduce(name):
            b, lib = bufs(name), libs[name]
            chk(lib.dal_canon_colsum_reduce(_ptr(b["parts"]), chunks, d, _ptr(b["cs"]), s), "dal_canon_colsum_reduce")

        for name in names:
            prep(name)
            bufs(name)["res"].zero_()
            resid(name)
            reduce(name)
        torch.cuda.synchronize()
        ref = out[names[0]]
        notes = []
        for name in names[1:]:
            bad = [k for k in ("ops", "norm", "parts", "acc", "res", "cs")
                   if not torch.equal(ref[k].view(torch.int64) if ref[k].dtype == torch.float64 else ref[k],
                                      out[name][k].view(torch.int64) if out[name][k].dtype == torch.float64
                                      else out[name][k])]
            notes.append(f"{name}: " + ("bits identical" if not bad else "DIFFERS in " + ",".join(bad)))
        reps = 10 if n * d < 5e7 else 3
        t = {(ph, name): [] for ph in ("prep", "resid", "reduce") for name in names}
        for _ in range(rounds):
            for ph, fn in (("prep", prep), ("resid", resid), ("reduce", reduce)):
                for name in names:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(reps):
                        fn(name)
                    e1.record()
                    torch.cuda.synchronize()
                    t[(ph, name)].append(e0.elapsed_time(e1) / reps * 1e3)
        for ph in ("prep", "resid", "reduce"):
            parts = [f"{name} {statistics.median(t[(ph, name)]):9.1f} us" for name in names]
            print(f"{n} x {d} {ph:6s}: " + " | ".join(parts), flush=True)
        print(f"{n} x {d}: " + "; ".join(notes), flush=True)
        del st, x, out, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
