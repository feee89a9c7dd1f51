"""A/B of the canonical column-sum partials kernel (DAL_COLSUM_FEAT features
per block), HIP events, same process, bits compared.  usage: python scripts/colsum_ab.py"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dal import engine  # noqa: E402
from dal._lib import DAL_CANON_CHUNK, call  # noqa: E402

dev = torch.device("cuda:0")
for n, d, dist in ((100_000, 64, "uniform"), (284_807, 30, "normal"), (2_000_000, 256, "uniform")):
    x = bench.upload(bench.host_pool(0, n, d, dist), dev)
    st = engine.PoolState(x, excluded=np.arange(10), device=dev)
    norm = st.norms()
    chunks = (n + DAL_CANON_CHUNK - 1) // DAL_CANON_CHUNK
    res, outs = {}, {}
    for rnd in range(6):
        for v in ("16", "8"):
            os.environ["DAL_COLSUM_FEAT"] = v
            p = torch.empty((chunks, d), dtype=torch.float64, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            call("dal_canon_colsum_partials", x.data_ptr(), n, d, d, norm.data_ptr(), st.flags.data_ptr(),
                 p.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                res.setdefault(v, []).append(e0.elapsed_time(e1) * 1e3)
            outs[v] = p
    for v in res:
        same = torch.equal(outs[v].view(torch.int64), outs["16"].view(torch.int64))
        print(f"n={n} d={d} features/block={v}: {np.median(res[v]):.1f} us identical={same}", flush=True)
