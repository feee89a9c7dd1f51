"""A/B timing of dal_max_cosine variants (interleaved rounds, one process;
outputs compared bitwise).  usage: python scripts/maxcos_ab.py [rounds]
env AB_VARIANTS: comma list of DAL_MAXCOS_VARIANT values ("32" = the
32x32x16 kernel; default a single variant); AB_ARG=1 times the arg-max form;
AB_NSHAPES limits the shapes."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "distributed-active-learning_amd"))
from dal import _lib  # noqa: E402
from dal.engine import _ptr, _stream  # noqa: E402
from dal.similarity import LabeledSet  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
variants = os.environ.get("AB_VARIANTS", "cur").split(",")
shapes = [(int(os.environ.get("AB_N", 8_000_000)), 128, 1024), (2_000_000, 64, 1000), (1_000_000, 256, 700)]
shapes = shapes[: int(os.environ.get("AB_NSHAPES", len(shapes)))]
dev = torch.device("cuda:0")
for n, d, m in shapes:
    g = torch.Generator(device=dev)
    g.manual_seed(n + d)
    x = torch.rand((n, d), generator=g, device=dev).to(torch.bfloat16)
    lab = LabeledSet(x[:m].clone(), dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    flops = 2.0 * n * lab.m * d
    res = {v: [] for v in variants}
    outs = {}
    for r in range(rounds + 1):
        for v in variants:
            os.environ["DAL_MAXCOS_VARIANT"] = v
            out = torch.empty(n, dtype=torch.float32, device=dev)
            arg = torch.empty(n, dtype=torch.int32, device=dev) if os.environ.get("AB_ARG") else None
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            _lib.call("dal_max_cosine", _ptr(x), n, d, _ptr(lab.rows), lab.m_pad, _ptr(lab.inv), 0,
                      _ptr(out), 0 if arg is None else _ptr(arg), _ptr(st), _stream(dev))
            e1.record()
            torch.cuda.synchronize()
            if r:
                res[v].append(e0.elapsed_time(e1))
            outs[v] = out
    same = all(torch.equal(outs[variants[0]], outs[v]) for v in variants)
    for v in variants:
        ms = float(np.median(res[v]))
        print(f"n={n} d={d} m={m} {v:4s} median {ms:8.3f} ms min {min(res[v]):8.3f}  "
              f"{flops / ms / 1e9:7.1f} TF/s  {100 * flops / ms / 1e9 / 2500:5.1f}% of 2.5 PF  "
              f"bitwise_same={same} max_abs_diff="
              f"{float((outs[v] - outs[variants[0]]).abs().max()):.3g}", flush=True)
