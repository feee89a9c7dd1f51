"""Why the bench's config-5 kernel time (10 back-to-back launches after the
selection steps) reads above the A/B script's (rounds of 5 launches): times
dal_max_cosine_unit at 8M x 128, m = 1,024 on the bench's pool (numpy
default_rng(0) uniform, host-generated) and on torch.rand data, with 5- and
10-launch windows, before and after 20 diversity-selection steps.
usage: python scripts/maxcos_window_probe.py"""
import os
import statistics
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from dal import _lib  # noqa: E402
from dal.engine import _ptr, _stream  # noqa: E402
from dal.similarity import LabeledSet, diversity_select  # noqa: E402

n, d, m, k = 8_000_000, 128, 1024, 1000
dev = torch.device("cuda:0")
pools = {
    "bench_pool": bench.upload(bench.host_pool(0, n, d, "uniform"), dev).to(torch.bfloat16),
    "torch_rand": torch.rand((n, d), device=dev, generator=torch.Generator(device=dev).manual_seed(0)).to(
        torch.bfloat16),
}
st = torch.zeros(1, dtype=torch.int32, device=dev)
out = torch.empty(n, dtype=torch.float32, device=dev)


def window(x, L, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        _lib.call("dal_max_cosine_unit", _ptr(x), n, d, _ptr(L.unit16), L.m_pad, _ptr(out), _ptr(st), _stream(dev))
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for phase in ("cold", "after_select"):
    for name, x in pools.items():
        L = LabeledSet(x[:m].clone(), dev)
        if phase == "after_select":
            cand = torch.arange(m, n, device=dev, dtype=torch.int64)
            for _ in range(20):
                diversity_select(x, None, k, candidates=cand, device=dev, labeled_rows=x[:m])
            torch.cuda.synchronize()
        for _ in range(2):
            window(x, L, 1)
        w5 = [window(x, L, 5) for _ in range(6)]
        w10 = [window(x, L, 10) for _ in range(3)]
        print(f"{phase:13s} {name:11s} 5-launch windows: median {statistics.median(w5):.4f} ms {['%.3f' % v for v in w5]}"
              f"  10-launch: {['%.3f' % v for v in w10]}", flush=True)
