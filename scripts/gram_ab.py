"""A/B timing of dal_gram_rowsum variants (interleaved rounds, one process).
usage: python scripts/gram_ab.py [rounds]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "distributed-active-learning_amd"))
from dal import _lib  # noqa: E402
from dal.engine import PoolState, _ptr, _stream  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
variants = os.environ.get("AB_VARIANTS", "single").split(",")
dev = torch.device("cuda:0")
shapes = [(100_000, 64), (500_000, 256), (200_000, 30)]
for n, d in shapes:
    g = torch.Generator(device=dev)
    g.manual_seed(n)
    x = torch.rand((n, d), generator=g, device=dev).clamp_(min=1e-7)
    st = PoolState(x, excluded=np.arange(10), device=dev)
    u, _ = st.normalized()
    flops = 2.0 * (n - 10) * (n - 10) * d
    res = {v: [] for v in variants}
    outs = {}
    for r in range(rounds + 1):
        for v in variants:
            os.environ["DAL_GRAM_VARIANT"] = v
            acc = torch.zeros(st.n_pad, dtype=torch.int64, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            _lib.call("dal_gram_rowsum", _ptr(u), st.n_pad, _ptr(u), st.n_pad, st.d_pad, st.d_pad,
                      _ptr(acc), 0, _stream(dev))
            e1.record()
            torch.cuda.synchronize()
            if r:
                res[v].append(e0.elapsed_time(e1))
            outs[v] = acc
    same = all(torch.equal(outs[variants[0]], outs[v]) for v in variants)
    for v in variants:
        ms = np.median(res[v])
        print(f"n={n} d={d} {v:7s} median {ms:9.3f} ms  min {min(res[v]):9.3f}  "
              f"{flops / ms / 1e9:7.1f} TF/s  {100 * flops / ms / 1e9 / 157.3:5.1f}%  bitwise_same={same}",
              flush=True)
