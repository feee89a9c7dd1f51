"""Same-process timing of the density Gram (dal_gram_rowsum_sym over every
column + dal_gram_sym_residual) with the in-tree library and the L-bits
variants of scripts/gram_lbits_build.py, interleaved; prints ms per density
call and the max relative density difference to the in-tree library.
usage: python scripts/gram_lbits_ab.py NxD M [M ...]"""
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
from dal.engine import PoolState  # noqa: E402

n, d = (int(v) for v in sys.argv[1].split("x"))
variants = ["tree"] + [f"lbits_{m}" for m in sys.argv[2:]]
dev = torch.device("cuda:0")
x = bench.upload(bench.host_pool(0, n, d, "uniform"), dev)
res = {}
dens = {}
for v in variants:
    _lib._LIB = None if hasattr(_lib, "_LIB") else None
res = {v: [] for v in variants}
states = {}
libpaths = {"tree": _lib.LIB_PATH}
for v in variants[1:]:
    libpaths[v] = os.path.join(REPO, "ab", v, "libdal.so")
orig = _lib.LIB_PATH
for rnd in range(3):
    for v in variants:
        _lib.LIB_PATH = libpaths[v]
        if hasattr(_lib, "_lib"):
            _lib._lib = None
        for attr in ("_LIB", "_handle", "_cached"):
            if hasattr(_lib, attr):
                setattr(_lib, attr, None)
        lib = _lib.load()
        st = PoolState(x, excluded=np.arange(10), device=dev)
        st.density_fixed()  # warm (prep + Gram)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        op = st.gram_operand()
        acc = torch.zeros(st.n_pad, dtype=torch.int64, device=dev)
        e0.record()
        for _ in range(2):
            acc.zero_()
            st.gram_accumulate(acc, op, st.n_pad)
            st.gram_residual(acc, op)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 2)
        dens[v] = acc[:n].double().cpu().numpy()
        del st, op
for v in variants:
    diff = np.nanmax(np.abs(dens[v][10:] - dens["tree"][10:]) / np.abs(dens["tree"][10:]))
    print(f"{v:10s} {statistics.median(res[v]):9.2f} ms/call  max rel diff vs tree {diff:.2e}", flush=True)
