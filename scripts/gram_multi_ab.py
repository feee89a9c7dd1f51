"""Same-process A/B of the density Gram call (dal_gram_rowsum_sym slices +
dal_gram_sym_residual, through PoolState) across several builds of libdal.so
(scripts/ab_build.sh), switched by rebinding dal._lib.  The accumulation is
exact integer arithmetic, so schedule-only variants must give identical
density bits (reported); then interleaved HIP-event timing of whole calls,
median and min over the rounds.

usage: python scripts/gram_multi_ab.py NAME=PATH [NAME=PATH ...] -- [NxD ...]
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
from dal.engine import PoolState  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    specs = [a.split("=", 1) for a in argv[:cut]]
    shapes = argv[cut + 1:] or ["284807x30", "100000x64"]
    libs = {name: bind(os.path.join(REPO, path) if not os.path.isabs(path) else path) for name, path in specs}
    names = list(libs)
    rounds = int(os.environ.get("AB_ROUNDS", "5"))
    dev = torch.device("cuda:0")
    for sh in shapes:
        n, d = (int(v) for v in sh.split("x"))
        _lib._lib = libs[names[0]]
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

        for name in names:
            run(name)
        torch.cuda.synchronize()
        bound = float(_lib._lib.dal_density_error_bound_sym(n - 10))
        notes = []
        for name in names[1:]:
            if not torch.equal(accs[names[0]], accs[name]):
                diff = float((accs[names[0]] - accs[name]).abs().max().item()) / 2.0 ** 32
                notes.append(f"{name} differs by <= {diff:.3g} (bound {bound:.3g})")
        reps = 5 if n * d < 5e7 else 1
        t = {name: [] for name in names}
        for _ in range(rounds):
            for name in names:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    run(name)
                e1.record()
                torch.cuda.synchronize()
                t[name].append(e0.elapsed_time(e1) / reps)
        fl = 2.0 * (n - 10) * (n - 10) * d
        parts = []
        for name in names:
            med = statistics.median(t[name])
            parts.append(f"{name} {med:.4f} ms ({fl / med / 1e9 / 2500:.4f}; min {min(t[name]):.4f})")
        print(f"{n} x {d}: " + " | ".join(parts) + ("  [" + "; ".join(notes) + "]" if notes else
                                                      "  [density bits identical]"), flush=True)
        _lib._lib = libs[names[0]]
        del st, x, op, accs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
