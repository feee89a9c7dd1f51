"""Host-side breakdown of the warm sharded step at P = 1 (real 1-rank RCCL
group): time spent in each phase of parallel.select's plan path (no extra
syncs; the status read is the step's one host wait), medians over many steps.
usage: python scripts/sharded_warm_breakdown.py [steps]"""
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
from dal import _lib, parallel  # noqa: E402
from dal.engine import _ptr, _stream  # noqa: E402
from dal.forest import Forest  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29557")
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
    parallel.select(sel, comm, unl, forest, k)
torch.cuda.synchronize()
lib = _lib.load()
T = {"launch": [], "all_gather": [], "merge_call": [], "status_read": [], "total": []}
for _ in range(steps):
    t0 = time.perf_counter()
    plan = sel.warm_plan(forest, k, 1.0)
    plan.launch(forest, unl)
    t1 = time.perf_counter()
    w = int(plan.packed.shape[0])
    g = comm.all_gather(plan.packed.reshape(1, w))
    t2 = time.perf_counter()
    buf = torch.empty(2 * k + 1, dtype=torch.int64, device=dev)
    st_or = buf[-1:].view(torch.int32)[:1]
    _lib.call("dal_topk_merge", _ptr(g), 1, w, k, 0, 0, _ptr(buf[:k]), _ptr(buf[k:2 * k]), 0, _ptr(st_or),
              _stream(dev))
    t3 = time.perf_counter()
    int(st_or.item())
    t4 = time.perf_counter()
    for key, a, b in (("launch", t0, t1), ("all_gather", t1, t2), ("merge_call", t2, t3), ("status_read", t3, t4),
                      ("total", t0, t4)):
        T[key].append((b - a) * 1e6)
for key, v in T.items():
    print(f"{key:12s} {statistics.median(v):8.1f} us")
t0 = time.perf_counter()
for _ in range(steps):
    parallel.select(sel, comm, unl, forest, k)
torch.cuda.synchronize()
print(f"select()     {(time.perf_counter() - t0) / steps * 1e6:8.1f} us/step")
dist.destroy_process_group()
