"""A/B: cold density step with the canonical column sum on a side stream
(default) vs serially on the main stream.  usage: python scripts/colsum_stream_ab.py"""
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np
import torch
from dal import engine
from dal.forest import Forest
import bench

dev = torch.device("cuda:0")
side_fn = engine._side_stream


def run(n, d, trees, mode, steps=40):
    engine._side_stream = side_fn if mode == "side" else (lambda device: torch.cuda.current_stream(device))
    x = bench.upload(bench.host_pool(0, n, d, "uniform"), dev)
    forest = Forest.synthetic(trees, 4, d, seed=1, dist="uniform")
    unl = torch.arange(10, n, device=dev, dtype=torch.int64)
    state = engine.PoolState(x, excluded=np.arange(10), device=dev)
    for _ in range(5):
        state.clear_caches()
        r = engine.density_step(state, unl, forest, 100)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        state.clear_caches()
        r = engine.density_step(state, unl, forest, 100)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print(f"n={n} d={d} T={trees} colsum={mode}: {ms:.4f} ms/step sel[:3]={r.indices[:3].tolist()}", flush=True)


for n, d, t in ((100000, 64, 10), (284807, 30, 100)):
    for rep in range(2):
        for mode in ("side", "main"):
            run(n, d, t, mode)
