"""Where a warm density step's wall time goes on the host (config 2 by
default): the whole engine.density_step call (what bench.py's warm latency
times), the WarmStepGraph.run call alone, and the bare dal_dw_plan_run C
call with preallocated outputs -- medians over 200 steps each.
usage: python scripts/warm_host_cost.py [NxD] [k]"""
import os
import statistics
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dal import engine  # noqa: E402
from dal.forest import Forest  # noqa: E402


def med(f, reps=200):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e6


def main():
    n, d = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "100000x64").split("x"))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    dev = torch.device("cuda:0")
    x = bench.upload(bench.host_pool(0, n, d, "uniform"), dev)
    forest = Forest.synthetic(10, 4, d, seed=1, dist="uniform")
    unl = torch.arange(10, n, device=dev, dtype=torch.int64)
    st = engine.PoolState(x, excluded=np.arange(10), device=dev)
    for _ in range(3):
        r = engine.density_step(st, unl, forest, k)
    torch.cuda.synchronize()
    (g,) = st._graphs.values()
    t_step = med(lambda: engine.density_step(st, unl, forest, k))
    t_run = med(lambda: g.run(forest, unl))
    lib = engine._lib.load()
    idx = torch.empty(k, dtype=torch.int64, device=dev)
    sc = torch.empty(k, dtype=torch.float64, device=dev)
    import ctypes

    status = ctypes.c_int32()
    ref = ctypes.byref(status)
    s = engine._raw_stream(dev)
    up, un, ip, sp = unl.data_ptr(), unl.shape[0], idx.data_ptr(), sc.data_ptr()
    t_c = med(lambda: lib.dal_dw_plan_run(g.plan, up, un, ip, sp, ref, s))
    t_empty = med(lambda: (torch.empty(k, dtype=torch.int64, device=dev), torch.empty(k, dtype=torch.float64,
                                                                                       device=dev)))
    print(f"{n}x{d} k={k}: density_step {t_step:.1f} us | WarmStepGraph.run {t_run:.1f} us | "
          f"dal_dw_plan_run {t_c:.1f} us | two torch.empty {t_empty:.1f} us", flush=True)
    del r


if __name__ == "__main__":
    main()
