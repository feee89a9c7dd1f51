"""Same-process timing of the two max-cosine kernels (K4): dal_max_cosine
(bf16 operands, per-column 1/||x_l|| scaling) vs dal_max_cosine_unit (fp16
folded unit labeled rows, max-only epilogue), interleaved, HIP events around
back-to-back launches on the launch stream; plus the max |difference|."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "distributed-active-learning_amd"))
from dal import _lib  # noqa: E402
from dal.similarity import LabeledSet  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream(dev).cuda_stream
for n, d, m in [(8_000_000, 128, 1024), (8_000_000, 64, 1024), (4_000_000, 256, 1024), (8_000_000, 128, 256)]:
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand((n, d), device=dev, generator=g).to(torch.bfloat16)
    L = LabeledSet(x[:m].clone(), dev)
    s = torch.zeros(1, dtype=torch.int32, device=dev)
    o1 = torch.empty(n, dtype=torch.float32, device=dev)
    o2 = torch.empty(n, dtype=torch.float32, device=dev)

    def k_bf16():
        _lib.call("dal_max_cosine", x.data_ptr(), n, d, L.rows.data_ptr(), L.m_pad, L.inv.data_ptr(), 0,
                  o1.data_ptr(), 0, s.data_ptr(), st)

    def k_unit():
        _lib.call("dal_max_cosine_unit", x.data_ptr(), n, d, L.unit16.data_ptr(), L.m_pad, o2.data_ptr(),
                  s.data_ptr(), st)

    res = {"bf16": [], "unit": []}
    for _ in range(2):
        k_bf16()
        k_unit()
    for _ in range(5):
        for name, fn in (("bf16", k_bf16), ("unit", k_unit)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 5)
    flops = 2.0 * n * m * d
    diff = (o1 - o2).abs().max().item()
    line = f"{n} x {d}, m={m}:"
    for name in ("bf16", "unit"):
        t = float(np.median(res[name]))
        line += f"  {name} {t:.4f} ms ({flops / t / 1e9 / 2500:.3f} of 2.5 PF)"
    print(line, f" max|bf16-unit| {diff:.2e} status {int(s.item())}", flush=True)
    del x, L, o1, o2
    torch.cuda.empty_cache()
