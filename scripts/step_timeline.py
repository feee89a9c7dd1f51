"""One cold config-2 density step, repeated, for a kernel timeline under
rocprofv3 --kernel-trace (analyse with scripts/step_timeline.py --analyse DIR).
usage: rocprofv3 --kernel-trace -d gpurun_out/tl -o tl --output-format csv -- python scripts/step_timeline.py [warm]
"warm": the density stays cached (the reference's per-iteration path); the
analysis then starts at the last step's mark_rows launch."""
import glob
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def analyse(d, first="normalize_split"):
    import csv
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[-1]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last step: from the last Gram launch's predecessor normalize_split
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    i0 = starts[-1]
    t0 = int(rows[i0]["Start_Timestamp"])
    prev_end = t0
    tot = 0
    for r in rows[i0:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("dal::(anonymous namespace)::", "").split("(")[0][-60:]
        print(f"{(s - t0) / 1e3:9.1f} us  gap {(s - prev_end) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  {name}")
        prev_end = e
        tot = e - t0
    print(f"step span {tot / 1e3:.1f} us")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "normalize_split")
        sys.exit(0)
    sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
    sys.path.insert(0, REPO)
    import numpy as np
    import torch
    from dal import engine
    from dal.forest import Forest
    import bench

    dev = torch.device("cuda:0")
    if len(sys.argv) > 2:  # step_timeline.py warm|cold CONFIG
        os.environ["TL_CONFIG"] = sys.argv[2]
    n, d = (int(v) for v in os.environ.get("TL_SHAPE", "100000x64").split("x"))
    trees, dist = 10, "uniform"
    if os.environ.get("TL_CONFIG"):  # a BASELINE config of bench.py (pool, forest)
        cfg = bench.CONFIGS[os.environ["TL_CONFIG"]]
        n, d, trees, dist = cfg["n"], cfg["d"], cfg["trees"], cfg["dist"]
    x = bench.upload(bench.host_pool(0, n, d, dist), dev)
    forest = Forest.synthetic(trees, 4, d, seed=1, dist=dist)
    unl = torch.arange(10, n, device=dev, dtype=torch.int64)
    state = engine.PoolState(x, excluded=np.arange(10), device=dev)
    warm = len(sys.argv) > 1 and sys.argv[1] == "warm"
    for _ in range(6):
        if not warm:
            state.clear_caches()
        r = engine.density_step(state, unl, forest, 100)
    torch.cuda.synchronize()
    print("ok", r.indices[:5].tolist())
