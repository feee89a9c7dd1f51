"""Run the fast-level-1 selection cases of tests/test_gpu_fast_select.py
through a given libdal.so build (a debug build prints its bound checks) and
compare with the oracle.  usage: python scripts/k3_debug_run.py LIB.so"""
import ctypes
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dal import _lib  # noqa: E402
from oracle import dal_oracle as O  # noqa: E402

lib = ctypes.CDLL(os.path.abspath(sys.argv[1]))
for name, (res, args) in _lib.SIGNATURES.items():
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = args
_lib._lib = lib
from dal import density_weighting as dw  # noqa: E402
from dal.engine import PoolState  # noqa: E402
from dal.forest import Forest  # noqa: E402

dev = torch.device("cuda:0")
for n, d, k in [(100_000, 64, 100), (20_000, 32, 10), (5_000, 48, 100), (250_000, 30, 1000)]:
    X = O.synthetic_pool(n, d, seed=0)
    of = O.synthetic_forest(10, 4, d, seed=1)
    E = np.arange(10)
    unl = np.arange(10, n)
    st = PoolState(X, excluded=E, device=dev)
    F = Forest.synthetic(10, 4, d, seed=1)
    _, ref_idx, ref_ss = O.density_select(X, unl, of, k, 1.0, E)
    for it in range(2):
        sel = dw.select(st, unl, F, k)
        torch.cuda.synchronize()
        ok = np.array_equal(sel.indices.cpu().numpy(), ref_idx) and np.array_equal(
            sel.selected_scores.cpu().numpy(), ref_ss)
        print(n, d, k, it, "match" if ok else "MISMATCH", flush=True)
