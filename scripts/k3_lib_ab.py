"""Same-process A/B of the standalone density-weighted selection (K3,
dal_dw_select through engine.dw_select_local) between two builds of
libdal.so: AB_BASE (default ab/k3_base/libdal.so) and the in-tree library,
switched by rebinding dal._lib between calls.  Per shape: selections
(indices + fp64 score bits) must be identical; then back-to-back calls
between two HIP events, interleaved A/B, median of the rounds.
usage: python scripts/k3_lib_ab.py [--base PATH] [--new PATH] [NxD[xT][:kK] ...]"""
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
from dal.forest import Forest  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        if not hasattr(lib, name):  # an older library: entry points added since
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


args = sys.argv[1:]
base = os.environ.get("AB_BASE", os.path.join(REPO, "ab", "k3_base", "libdal.so"))
new = _lib.LIB_PATH
while args[:1] in (["--base"], ["--new"]):  # (--base instead of AB_BASE; --new instead of the in-tree library)
    path = args[1] if os.path.isabs(args[1]) else os.path.join(REPO, args[1])
    if args[0] == "--base":
        base = path
    else:
        new = path
    args = args[2:]
libs = {"base": bind(base), "new": bind(new)}
dev = torch.device("cuda:0")
for spec in args or ["100000x64", "2000000x256", "284807x30x100", "2000000x256:k1000"]:
    sh, _, kk = spec.partition(":k")
    K = int(kk) if kk else 100
    parts = [int(v) for v in sh.split("x")]
    n, d = parts[:2]
    trees = parts[2] if len(parts) > 2 else 10
    _lib._lib = libs["new"]
    x = bench.upload(bench.host_pool(0, n, d, "normal" if d == 30 else "uniform"), dev)
    forest = Forest.synthetic(trees, 4, d, seed=1)
    st = engine.PoolState(x, excluded=np.arange(10), device=dev)
    dens = st.density_fixed()
    flags, _, _ = st.row_flags(torch.arange(10, n, device=dev))
    lut = engine.device_lut("entropy", trees, dev)
    votes, scores, klo, khi = engine.forest_score(st, forest, lut, flags, DAL_DESCENDING, density=dens,
                                                  density_err=engine.density_error(st), want_hi=True)
    cs = st.colsum()
    torch.cuda.synchronize()
    res, t = {}, {"base": [], "new": []}
    for name in ("base", "new"):
        _lib._lib = libs[name]
        idx, sc, _ = engine.dw_select_local(st, flags, votes, klo, khi, lut, K, 1.0, cs)
        res[name] = (idx.cpu().numpy(), sc.cpu().numpy())
    same = np.array_equal(res["base"][0], res["new"][0]) and np.array_equal(
        res["base"][1].view(np.int64), res["new"][1].view(np.int64))
    for _ in range(7):
        for name in ("base", "new"):
            _lib._lib = libs[name]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                engine.dw_select_local(st, flags, votes, klo, khi, lut, K, 1.0, cs, sync=False)
            e1.record()
            torch.cuda.synchronize()
            t[name].append(e0.elapsed_time(e1) / 20 * 1000)
    print(f"{n} x {d} x T{trees} k={K}: base {statistics.median(t['base']):.1f} us  new {statistics.median(t['new']):.1f} us"
          f"  {'selection identical' if same else 'SELECTION DIFFERS'}", flush=True)
    _lib._lib = libs["new"]
    del st, x
    torch.cuda.empty_cache()
