"""Timing ablations of the symmetric Gram kernel (results of the ablated
builds are WRONG by construction; timing only): build/abl1 = no column-sum
epilogue, build/abl2 = no stage DMA.  usage: python scripts/gram_ablate.py"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
from dal import _lib  # noqa: E402
from dal.engine import PoolState, _ptr, _stream  # noqa: E402

dev = torch.device("cuda:0")
libs = {"full": _lib.load()}
for a in os.environ.get("AB_LIBS", "abl1,abl2").split(","):
    p = os.path.join(REPO, os.environ.get("AB_DIR", "build"), a, "libdal.so")
    if os.path.exists(p):
        libs[a] = ctypes.CDLL(p)
# variants of the current library selected by environment knobs: name=VAR:VAL
knobs = [k.split("=") for k in os.environ.get("AB_KNOBS", "").split(",") if k]
for name, kv in knobs:
    libs[name] = (libs["full"], kv)
SHAPES = [tuple(int(v) for v in t.split("x")) for t in os.environ.get("AB_SHAPES", "100000x64,200000x30").split(",")]
ROUNDS = int(os.environ.get("AB_ROUNDS", "4"))
for n, d in SHAPES:
    g = torch.Generator(device=dev)
    g.manual_seed(n)
    x = torch.rand((n, d), generator=g, device=dev).clamp_(min=1e-7)
    st = PoolState(x, excluded=np.arange(10), device=dev, gram="sym")
    sp = st.gram_operand()
    nb = st.n_pad // 256
    res = {k: [] for k in libs}
    for r in range(ROUNDS):
        for k, L in libs.items():
            if isinstance(L, tuple):
                L, kv = L
                var, val = kv.split(":")
                os.environ[var] = val
            else:
                for _, kv in knobs:
                    os.environ.pop(kv.split(":")[0], None)
            acc = torch.zeros(st.n_pad, dtype=torch.int64, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            rc = L.dal_gram_rowsum_sym(ctypes.c_void_p(_ptr(sp)), ctypes.c_int64(0), ctypes.c_int64(nb),
                                       ctypes.c_void_p(_ptr(sp)), ctypes.c_int64(0), ctypes.c_int64(0),
                                       ctypes.c_int64(nb), ctypes.c_int64(nb), ctypes.c_int64(st.d_pad),
                                       ctypes.c_void_p(_ptr(acc)), 0, ctypes.c_void_p(_stream(dev)))
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0
            if r:
                res[k].append(e0.elapsed_time(e1))
    for k in libs:
        print(f"n={n} d={d} {k:5s} median {np.median(res[k]):.3f} ms", flush=True)
