"""Wall-clock breakdown of the warm config-2 density step (density cached,
hipGraph replay): host time before the replay is queued, replay -> status
read (dal_dw_plan_run: the GPU span + the sync), and the rest of the step.  Prints medians
over many steps.  usage: python scripts/warm_breakdown.py [n x d]"""
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

dev = torch.device("cuda:0")
n, d = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "100000x64").split("x"))
x = bench.upload(bench.host_pool(0, n, d, "uniform"), dev)
forest = Forest.synthetic(10, 4, d, seed=1, dist="uniform")
unl = torch.arange(10, n, device=dev, dtype=torch.int64)
state = engine.PoolState(x, excluded=np.arange(10), device=dev)
engine.density_step(state, unl, forest, 100)  # cold
for _ in range(20):
    engine.density_step(state, unl, forest, 100)
torch.cuda.synchronize()

marks = {}
orig_run = engine.WarmStepGraph.run


def run(self, *a):
    marks["pre"] = time.perf_counter()
    r = orig_run(self, *a)
    marks["synced"] = time.perf_counter()
    return r


engine.WarmStepGraph.run = run
rows = []
for _ in range(300):
    marks.clear()
    t0 = time.perf_counter()
    sel = engine.density_step(state, unl, forest, 100)
    t1 = time.perf_counter()
    rows.append((marks["pre"] - t0, marks["synced"] - marks["pre"], t1 - marks["synced"], t1 - t0))
torch.cuda.synchronize()
med = [statistics.median(c) * 1e6 for c in zip(*rows)]
print(f"warm step {n}x{d} (median of {len(rows)}, us): host before the plan call {med[0]:.1f}, "
      f"WarmStepGraph.run (outputs + dal_dw_plan_run: refresh, replay, sync) {med[1]:.1f}, after {med[2]:.1f}, total {med[3]:.1f}")
t = time.perf_counter()
for _ in range(200):
    sel = engine.density_step(state, unl, forest, 100)
torch.cuda.synchronize()
print(f"plain loop: {(time.perf_counter() - t) / 200 * 1e6:.1f} us/step")
