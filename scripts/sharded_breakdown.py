"""Where the warm sharded step's time goes (P = 1, real RCCL group): each
phase of parallel.select timed with a device sync after it (the syncs add
their own ~10 us each; the sum is an upper bound of the step).
usage: python scripts/sharded_breakdown.py [steps]"""
import os
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
from bench import host_pool, upload  # noqa: E402
from dal import engine, parallel  # noqa: E402
from dal.forest import Forest  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29556")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
n, d, k = 100_000, 64, 100
x = upload(host_pool(0, n, d, "uniform"), dev)
forest = Forest.synthetic(10, 4, d, seed=1)
unl = torch.arange(10, n, device=dev, dtype=torch.int64)
sel = parallel.ShardedSelector(x, n, 0, 1, excluded=np.arange(10), device=dev)
comm = parallel.TorchComm()
for _ in range(5):
    parallel.select(sel, comm, unl, forest, k, mode="dw")
torch.cuda.synchronize()

T = {}


def mark(name, t0):
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    T.setdefault(name, []).append((t1 - t0) * 1e6)
    return t1


for _ in range(steps):
    t = time.perf_counter()
    u = sel.index_tensor(unl)
    t = mark("index_tensor", t)
    top = sel.local_select(None, sel._parts_full, u, forest, k, "dw")
    t = mark("local_select (flags + fused step)", t)
    g = parallel.gather_topk(comm, top, sel.status_word())
    t = mark("gather_topk (pack + all-gather + unpack)", t)
    out = parallel.merge_topk(*g[:3], k, parallel.hip_sort_positions, all_valid=True)
    t = mark("merge_topk", t)
    st = 0
    for v in g[3].tolist():
        st |= int(v)
    t = mark("status read", t)
tot = 0.0
for name, v in T.items():
    m = statistics.median(v)
    tot += m
    print(f"{name:42s} {m:7.1f} us", flush=True)
print(f"{'sum':42s} {tot:7.1f} us")
t0 = time.perf_counter()
for _ in range(steps):
    parallel.select(sel, comm, unl, forest, k, mode="dw")
torch.cuda.synchronize()
print(f"select() unperturbed: {(time.perf_counter() - t0) / steps * 1e6:.1f} us/step")
dist.destroy_process_group()
