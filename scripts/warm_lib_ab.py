"""Same-process A/B of the warm density-weighted step (the hipGraph plan:
mark -> fused forest score + group minima -> select) between two builds of
libdal.so: AB_BASE (default: the in-tree library) and AB_NEW, switched by
rebinding dal._lib; one PoolState per library (each computes its density
once).  Selections (indices + fp64 score bits) must be identical; then
interleaved wall timing of warm steps (host included, as a user runs them).
usage: AB_NEW=path python scripts/warm_lib_ab.py [CONFIG ...]
       python scripts/warm_lib_ab.py --base PATH --new PATH [CONFIG ...]"""
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
from dal import _lib, engine  # noqa: E402
from dal.forest import Forest  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


args = sys.argv[1:]
paths = {"base": os.environ.get("AB_BASE", _lib.LIB_PATH), "new": os.environ.get("AB_NEW")}
while args[:1] in (["--base"], ["--new"]):
    paths[args[0][2:]] = args[1] if os.path.isabs(args[1]) else os.path.join(REPO, args[1])
    args = args[2:]
libs = {name: bind(path) for name, path in paths.items()}
dev = torch.device("cuda:0")
for c in args or ["4", "2"]:
    cfg = bench.CONFIGS[c]
    n, d, trees, dist = cfg["n"], cfg["d"], cfg["trees"], cfg["dist"]
    x = bench.upload(bench.host_pool(0, n, d, dist), dev)
    forest = Forest.synthetic(trees, 4, d, seed=1, dist=dist)
    unl = torch.arange(10, n, device=dev, dtype=torch.int64)
    states, sel = {}, {}
    for name in ("base", "new"):
        _lib._lib = libs[name]
        states[name] = engine.PoolState(x, excluded=np.arange(10), device=dev)
        engine.density_step(states[name], unl, forest, 100)
        r = engine.density_step(states[name], unl, forest, 100)
        sel[name] = (r.indices.cpu().numpy(), r.selected_scores.cpu().numpy())
    same = np.array_equal(sel["base"][0], sel["new"][0]) and np.array_equal(
        sel["base"][1].view(np.int64), sel["new"][1].view(np.int64))
    t = {"base": [], "new": []}
    for _ in range(7):
        for name in ("base", "new"):
            _lib._lib = libs[name]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                engine.density_step(states[name], unl, forest, 100)
            torch.cuda.synchronize()
            t[name].append((time.perf_counter() - t0) / 20 * 1e6)
    print(f"config {c}: warm step base {statistics.median(t['base']):.1f} us  new {statistics.median(t['new']):.1f} us"
          f"  {'selection identical' if same else 'SELECTION DIFFERS'}", flush=True)
    _lib._lib = libs["base"]
    del states, x
    torch.cuda.empty_cache()
