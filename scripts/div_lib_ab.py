"""Same-process A/B of the whole batch-mode diversity selection (config 5:
dal.similarity.diversity_select -- labeled-set prep, dal_max_cosine_unit,
candidate marking, interval keys, the exact selection with its fp64 re-rank)
between two builds of libdal.so, switched by rebinding dal._lib.  The
selections (indices + fp64 score bits) must be identical; then interleaved
wall timing of whole calls (host included, as the bench's step runs them).
usage: python scripts/div_lib_ab.py --base PATH [--new PATH] [NxDxM]"""
import ctypes
import os
import statistics
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dal import _lib  # noqa: E402
from dal.similarity import diversity_select  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


args = sys.argv[1:]
paths = {"base": None, "new": _lib.LIB_PATH}
while args[:1] in (["--base"], ["--new"]):
    paths[args[0][2:]] = args[1] if os.path.isabs(args[1]) else os.path.join(REPO, args[1])
    args = args[2:]
libs = {name: bind(p) for name, p in paths.items()}
cfg = bench.CONFIGS["5"]
n, d, m, k = cfg["n"], cfg["d"], cfg["m"], cfg["k"]
if args:
    n, d, m = (int(v) for v in args[0].split("x"))
dev = torch.device("cuda:0")
x = bench.upload(bench.host_pool(0, n, d, cfg["dist"]), dev).to(torch.bfloat16)
lab = x[:m].clone()
cand = torch.arange(m, n, device=dev, dtype=torch.int64)
sel = {}
for name, lib in libs.items():
    _lib._lib = lib
    s = diversity_select(x, None, k, candidates=cand, device=dev, labeled_rows=lab)
    sel[name] = (s.indices.cpu().numpy(), s.selected_scores.cpu().numpy())
same = np.array_equal(sel["base"][0], sel["new"][0]) and np.array_equal(
    sel["base"][1].view(np.int64), sel["new"][1].view(np.int64))
t = {name: [] for name in libs}
for _ in range(7):
    for name, lib in libs.items():
        _lib._lib = lib
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            diversity_select(x, None, k, candidates=cand, device=dev, labeled_rows=lab)
        torch.cuda.synchronize()
        t[name].append((time.perf_counter() - t0) / 10 * 1e3)
print(f"{n} x {d}, m={m}, k={k}: diversity_select base {statistics.median(t['base']):.4f} ms  "
      f"new {statistics.median(t['new']):.4f} ms  {'selection identical' if same else 'SELECTION DIFFERS'}",
      flush=True)
