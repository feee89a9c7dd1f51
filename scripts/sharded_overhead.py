"""Fixed per-step cost of the sharded (multi-GPU) selection path, measured on
ONE GPU with a world-size-1 RCCL process group: the same collectives and
launches as every rank runs at N > 1, against the single-GPU step.
usage: python scripts/sharded_overhead.py [steps]"""
import os
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

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29555")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
n, d, k = 100_000, 64, 100
x = upload(host_pool(0, n, d, "uniform"), dev)
forest = Forest.synthetic(10, 4, d, seed=1)
E = np.arange(10)
unl = torch.arange(10, n, device=dev, dtype=torch.int64)
sel = parallel.ShardedSelector(x, n, 0, 1, excluded=E, device=dev)
comm = parallel.TorchComm()
st = engine.PoolState(x, excluded=E, device=dev)


def sharded():
    sel.clear_caches()
    return parallel.select(sel, comm, unl, forest, k, mode="dw")


def single():
    st.clear_caches()
    r = engine.density_step(st, unl, forest, k)
    return r.indices, r.selected_scores


def single_warm():
    r = engine.density_step(st, unl, forest, k)
    return r.indices, r.selected_scores


def sharded_warm():  # density cached: one fused dal_dw_step per rank
    return parallel.select(sel, comm, unl, forest, k, mode="dw")


def sharded_warm_sep():  # the same with K2 and K3 as separate calls (event-timed path)
    sel.state.forest_events, sel.state.select_events = [], []
    r = parallel.select(sel, comm, unl, forest, k, mode="dw")
    sel.state.forest_events = sel.state.select_events = None
    return r


for name, fn in (("single", single), ("sharded-P1", sharded), ("single", single), ("sharded-P1", sharded),
                 ("single-warm", single_warm), ("sh-warm-fused", sharded_warm), ("sh-warm-sep", sharded_warm_sep),
                 ("sh-warm-fused", sharded_warm), ("sh-warm-sep", sharded_warm_sep)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        idx, sc = fn()
    torch.cuda.synchronize()
    print(f"{name:14s} {1000 * (time.perf_counter() - t0) / steps:.3f} ms/step", flush=True)
a = single()
b = sharded()
c = sharded_warm()
print("same selection:", bool(torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[0], c[0])
                              and torch.equal(a[1], c[1])), flush=True)
dist.destroy_process_group()
