"""Phase timing of summary_select_kernel (the fast level 1 of dal_dw_step)
from a trace build (-DDAL_K3_TRACE: s_memrealtime stamps, 10 ns ticks, in a
device array read by dal_k3_trace).  usage: python scripts/k3_trace.py LIB NxD [trees] [k]"""
import ctypes
import os
import statistics
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dal import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
import bench  # noqa: E402
from dal import engine  # noqa: E402
from dal.forest import Forest  # noqa: E402

dev = torch.device("cuda:0")
n, d = (int(v) for v in sys.argv[2].split("x"))
trees = int(sys.argv[3]) if len(sys.argv) > 3 else 10
k = int(sys.argv[4]) if len(sys.argv) > 4 else 100
lib = _lib.load()
lib.dal_k3_trace.argtypes = [ctypes.c_void_p]
lib.dal_k3_trace_reset.argtypes = []
x = bench.upload(bench.host_pool(0, n, d, "normal" if d == 30 else "uniform"), dev)
st = engine.PoolState(x, excluded=np.arange(10), device=dev)
forest = Forest.synthetic(trees, 4, d, seed=1)
lut = engine.device_lut("entropy", trees, dev)
flags, _, _ = st.row_flags(torch.arange(10, n, device=dev))
dens, cs = st.density_fixed(), st.colsum()
buf = (ctypes.c_ulonglong * 1024)()
rows = []
for it in range(30):
    engine.dw_step_local(st, forest, flags, dens, lut, k, 1.0, cs)
    torch.cuda.synchronize()
    lib.dal_k3_trace(ctypes.addressof(buf))
    t = list(buf)
    G = t[5]
    arr = [t[256 + b] for b in range(G)]
    t0 = t[0]
    rows.append(((t[10] - t0) / 100, (t[11] - t0) / 100, t[13], (t[1] - t0) / 100, (t[2] - t0) / 100, (min(arr) - t0) / 100, (max(arr) - t0) / 100,
                 (t[3] - t0) / 100, (t[7] - t0) / 100, (t[8] - t0) / 100, (t[9] - t0) / 100, (t[6] - t0) / 100,
                 t[4], G, sum(t[512 + b] for b in range(G)), t[20] / 100, t[21] / 100, t[22] / 100, t[23],
                 (t[14] - t0) / 100, (t[16] - t0) / 100, (t[17] - t0) / 100, t[15],
                 t[24] / 100, t[25] / 100, t[26] / 100))
    lib.dal_k3_trace_reset()
print(f"{n}x{d} T={trees} k={k} level1_fast={st.level1_fast} (us from block 0's start; medians of 30)")
names = ["minmax", "passes_done", "bucket", "tau", "hits", "first_arrive", "last_arrive", "sort_start", "sort_read_hdr", "sort_loaded", "sort_ranked",
         "end", "cands", "grid", "hit_groups", "max_scan", "max_score", "max_store_drain", "max_block_cands",
         "rank_cleared", "sel_compacted", "sel_sorted", "sel_m",
         "max_sc_loads", "max_sc_divs", "max_sc_sum"]  # (the last three: K3_TRACE_SCORE=1 builds only)
for j, nm in enumerate(names):
    print(f"  {nm:13s} {statistics.median(r[j] for r in rows[5:]):9.2f}")
