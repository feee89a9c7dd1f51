"""A/B of the fp32-MFMA Gram row-sum (dal_gram_rowsum) against the split-fp16
one (dal_gram_rowsum_split): time, agreement with the canonical fp64 density
(separable form), the rigorous bounds, and grid-size invariance of the split
kernel.  usage: python scripts/gram_split_ab.py [rounds]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "distributed-active-learning_amd"))
from dal import _lib  # noqa: E402
from dal.engine import PoolState, _ptr, _stream  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
shapes = [(s.split("x")) for s in os.environ.get("AB_SHAPES", "100000x64,200000x30,500000x256").split(",")]
dev = torch.device("cuda:0")
lib = _lib.load()
for n, d in [(int(a), int(b)) for a, b in shapes]:
    g = torch.Generator(device=dev)
    g.manual_seed(n)
    x = torch.rand((n, d), generator=g, device=dev).clamp_(min=1e-7)
    st = PoolState(x, excluded=np.arange(10), device=dev)
    u, _ = st.normalized()
    sp = torch.empty(int(lib.dal_split_f16_halves(st.n_pad, st.d_pad)), dtype=torch.int16, device=dev)
    _lib.call("dal_split_f16", _ptr(u), st.n_pad, st.d_pad, st.d_pad, _ptr(sp), _stream(dev))
    flops = 2.0 * (n - 10) * (n - 10) * d
    kinds = os.environ.get("AB_KINDS", "f32,split").split(",")
    t = {k: [] for k in kinds}
    accs = {}

    def run(kind, grid=0):
        acc = torch.zeros(st.n_pad, dtype=torch.int64, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        os.environ["DAL_GRAM_SCHED"] = "0" if kind.endswith("s0") else "1"
        os.environ["DAL_GRAM_MT"] = "32" if "32" in kind else "16"
        # sym: default kernel; symk1: 256-row-block kernel; symsgN: its epilogue variant N
        os.environ.pop("DAL_GRAM_SG", None)
        os.environ.pop("DAL_GRAM_SYM", None)
        if kind.startswith("symsg"):
            os.environ["DAL_GRAM_SYM"] = "1"
            os.environ["DAL_GRAM_SG"] = kind[5:]
        elif kind in ("symk1", "symk2"):
            os.environ["DAL_GRAM_SYM"] = kind[-1]
        if kind.startswith("sym"):
            nb = st.n_pad // 256
            _lib.call("dal_gram_rowsum_sym", _ptr(sp), 0, nb, _ptr(sp), 0, 0, nb, nb, st.d_pad,
                      _ptr(acc), grid, _stream(dev))
        elif kind == "f32":
            _lib.call("dal_gram_rowsum", _ptr(u), st.n_pad, _ptr(u), st.n_pad, st.d_pad, st.d_pad,
                      _ptr(acc), grid, _stream(dev))
        else:
            _lib.call("dal_gram_rowsum_split", _ptr(sp), st.n_pad, _ptr(sp), st.n_pad, st.d_pad,
                      _ptr(acc), grid, _stream(dev))
        e1.record()
        torch.cuda.synchronize()
        return acc, e0.elapsed_time(e1)

    for r in range(rounds + 1):
        for kind in kinds:
            acc, ms = run(kind)
            if r:
                t[kind].append(ms)
            accs[kind] = acc
    canon = st.density_exact()[10:n]
    for kind in kinds:
        dk = accs[kind][10:n].to(torch.float64) / 2.0**32
        err = (dk - canon).abs()
        bound = (lib.dal_density_error_bound if kind.startswith("f32") else
                 lib.dal_density_error_bound_sym if kind.startswith("sym") else lib.dal_density_error_bound_split)(n - 10)
        ms = float(np.median(t[kind]))
        print(f"n={n} d={d} {kind:6s} median {ms:8.3f} ms  {flops / ms / 1e9:7.1f} TF/s "
              f"({100 * flops / ms / 1e9 / 157.3:5.1f}% of fp32 peak)  max|err| {float(err.max()):.3e} "
              f"max rel {float((err / canon.abs()).max()):.3e}  bound {bound:.3e}  "
              f"within={bool(float(err.max()) <= bound)}", flush=True)
    sk = [k for k in kinds if k.startswith("split")]
    for kk in [k for k in kinds if k.startswith("symsg")]:
        if "sym" in kinds:
            print(f"   sym vs {kk}: same bits {torch.equal(accs['sym'], accs[kk])}, max |diff| "
                  f"{int((accs['sym'] - accs[kk]).abs().max())} (2^-32 units)", flush=True)
    for kk in [k for k in kinds if k.startswith("sym")]:
        a2, _ = run(kk, grid=37)
        a3, _ = run(kk, grid=1000)
        print(f"   {kk} grid-invariant: {torch.equal(a2, accs[kk]) and torch.equal(a3, accs[kk])}",
              flush=True)
    if len(sk) > 1:
        print(f"   all split variants same bits: {all(torch.equal(accs[sk[0]], accs[k]) for k in sk)}",
              flush=True)
    if "split" not in kinds:
        continue
    a2, _ = run("split", grid=37)
    a3, _ = run("split", grid=1000)
    print(f"   split grid-invariant: {torch.equal(a2, accs['split']) and torch.equal(a3, accs['split'])}",
          flush=True)
    del sp, st, u, x
    torch.cuda.empty_cache()
