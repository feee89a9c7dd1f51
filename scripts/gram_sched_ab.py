"""Same-process A/B of the density Gram call (dal_gram_rowsum_sym slices +
dal_gram_sym_residual, through PoolState) between two builds of libdal.so:
AB_BASE (default ab/gram_base/libdal.so) and AB_NEW (default the in-tree
library), switched by rebinding dal._lib.  The accumulation is exact integer
arithmetic, so the densities must be bit-identical; then interleaved HIP-event
timing of whole calls, median of the rounds.
usage: python scripts/gram_sched_ab.py [NxD ...]   (d = 30: config 3's N(0,1) pool)"""
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


def bind(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


libs = {"base": bind(os.environ.get("AB_BASE", os.path.join(REPO, "ab", "gram_base", "libdal.so"))),
        "new": bind(os.environ.get("AB_NEW", _lib.LIB_PATH))}
dev = torch.device("cuda:0")
for sh in sys.argv[1:] or ["284807x30", "100000x64"]:
    n, d = (int(v) for v in sh.split("x"))
    _lib._lib = libs["new"]
    x = bench.upload(bench.host_pool(0, n, d, "normal" if d == 30 else "uniform"), dev)
    st = PoolState(x, excluded=np.arange(10), device=dev)
    op = st.gram_operand()
    accs = {}

    def run(name):
        _lib._lib = libs[name]
        acc = accs.setdefault(name, torch.zeros(st.n_pad, dtype=torch.int64, device=dev))
        acc.zero_()
        st.gram_accumulate(acc, op, st.n_pad)
        st.gram_residual(acc, op)

    for name in ("base", "new"):
        run(name)
    torch.cuda.synchronize()
    same = torch.equal(accs["base"], accs["new"])
    # fixed point in units of 2^-32: the largest density difference, against the rigorous bound
    diff = float((accs["base"] - accs["new"]).abs().max().item()) / 2.0 ** 32
    bound = float(_lib._lib.dal_density_error_bound_sym(n - 10))
    reps = 5 if n * d < 5e7 else 2
    t = {"base": [], "new": []}
    for _ in range(5):
        for name in ("base", "new"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run(name)
            e1.record()
            torch.cuda.synchronize()
            t[name].append(e0.elapsed_time(e1) / reps)
    fl = 2.0 * (n - 10) * (n - 10) * d
    tb, tn = statistics.median(t["base"]), statistics.median(t["new"])
    print(f"{n} x {d}: base {tb:.4f} ms ({fl / tb / 1e9 / 2500:.3f})  new {tn:.4f} ms ({fl / tn / 1e9 / 2500:.3f})  "
          f"{'density bits identical' if same else f'densities differ by <= {diff:.3g} (bound {bound:.3g})'}",
          flush=True)
    _lib._lib = libs["new"]
    del st, x, op, accs
    torch.cuda.empty_cache()
