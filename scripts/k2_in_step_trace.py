"""K2 inside a warm step vs alone, one process, for rocprofv3 --kernel-trace:
5 standalone dal_forest_score_blocked launches (no hooks), 5 eager fused
steps (dal_dw_step: group-minima fold, stored row flags), 5 warm-plan
replays (hipGraph: the fold plus the stamp-derived row flags), 5 eager steps
with the exact level 1 (no fold).  Analyse with
--analyse DIR: per kernel name and phase, the median duration.
usage: [K2_LIB=path] python scripts/k2_in_step_trace.py [CONFIG]   |   --analyse DIR"""
import glob
import os
import statistics
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def analyse(d):
    """The blocked K2 launches in order: 5 alone, 5 in eager steps, 6 in plan
    replays, 5 in eager steps with the exact level 1 (no group-minima hooks)."""
    import csv
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[-1]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    k2 = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
          if "forest_blocked_kernel" in r["Kernel_Name"]]
    sel = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
           if "summary_select_kernel" in r["Kernel_Name"]]
    for nm, a, b in (("alone", 0, 5), ("eager step", 5, 10), ("plan replay", 10, 16), ("exact L1", 16, 21)):
        if len(k2) < b:
            continue
        print(f"K2 {nm:12s} median {statistics.median(k2[a:b]):8.1f} us  {[round(v, 1) for v in k2[a:b]]}")
    print(f"selection launches (cold, eager x5, plan x6): {[round(v, 1) for v in sel]}")


def main():
    sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
    sys.path.insert(0, REPO)
    import numpy as np
    import torch

    from dal import _lib
    if os.environ.get("K2_LIB"):  # an A/B build in place of the product library
        _lib.LIB_PATH = os.path.abspath(os.environ["K2_LIB"])
    import bench
    from dal import engine
    if os.environ.get("DAL_AB_LIB"):  # an A/B build in place of the product library
        import ctypes

        lib = ctypes.CDLL(os.path.abspath(os.environ["DAL_AB_LIB"]))
        for name, (res, args) in _lib.SIGNATURES.items():
            getattr(lib, name).restype = res
            getattr(lib, name).argtypes = args
        _lib._lib = lib
    from dal._lib import DAL_DESCENDING
    from dal.forest import Forest

    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "4"]
    n, d = cfg["n"], cfg["d"]
    dev = torch.device("cuda:0")
    x = bench.upload(bench.host_pool(0, n, d, cfg["dist"]), dev)
    forest = Forest.synthetic(cfg["trees"], cfg["depth"], d, seed=1, dist=cfg["dist"])
    unl = torch.arange(10, n, device=dev, dtype=torch.int64)
    st = engine.PoolState(x, excluded=np.arange(10), device=dev)
    engine.density_step(st, unl, forest, cfg["k"])  # cold
    xb = st.blocked_pool(forest)
    dens = st.density_fixed()
    flags, _, _ = st.row_flags(unl)
    lut = engine.device_lut("entropy", forest.n_trees, dev)
    torch.cuda.synchronize()
    for _ in range(5):
        engine.forest_score(st, forest, lut, flags, DAL_DESCENDING, density=dens,
                            density_err=engine.density_error(st), want_hi=True, xb=xb)
    torch.cuda.synchronize()
    st.use_graphs = False
    for _ in range(5):
        engine.density_step(st, unl, forest, cfg["k"])
    torch.cuda.synchronize()
    st.use_graphs = True
    for _ in range(6):
        engine.density_step(st, unl, forest, cfg["k"])
    torch.cuda.synchronize()
    # eager steps with the exact level 1 (no group-minima hooks in the score kernel)
    st.use_graphs, st.level1_fast = False, False
    for _ in range(5):
        engine.density_step(st, unl, forest, cfg["k"])
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
    else:
        main()
