"""Same-process A/B of the symmetric Gram's scheduling knobs (DAL_GRAM_NC
column-chunk count, DAL_GRAM_CONTIG) on large shapes: time per full density
(every 64-feature slice) and bit equality of the fixed-point row sums.
usage: AB_SHAPES=2000000x256 AB_VARIANTS="default,NC=2,CONTIG=1" python scripts/gram_knob_ab.py [rounds]"""
import os
import statistics
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from dal import engine  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
variants = os.environ.get("AB_VARIANTS", "default,NC=1,NC=2,NC=4,NC=8,CONTIG=1").split(",")
dev = torch.device("cuda:0")
for shape in os.environ.get("AB_SHAPES", "1000000x256").split(","):
    n, d = (int(v) for v in shape.split("x"))
    x = bench.upload(bench.host_pool(0, n, d, "uniform"), dev)
    st = engine.PoolState(x, excluded=np.arange(10), device=dev)
    flops = 2.0 * (n - 10) * (n - 10) * d
    times = {v: [] for v in variants}
    ref = None
    for r in range(rounds + 1):
        for v in variants:
            for key in ("DAL_GRAM_NC", "DAL_GRAM_NC_MIN", "DAL_GRAM_CONTIG", "DAL_GRAM_ANT"):
                os.environ.pop(key, None)
            if v != "default":
                for part in v.split("+"):  # e.g. CONTIG=0+NC=32
                    kk, val = part.rsplit("=", 1)
                    os.environ["DAL_GRAM_" + kk] = val
            st.clear_caches()
            st.gram_operand()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            dens = st.density_fixed()
            b.record()
            torch.cuda.synchronize()
            if r:
                times[v].append(a.elapsed_time(b))
            if ref is None:
                ref = dens.clone()
            elif not torch.equal(dens, ref):
                print(f"{shape} {v}: BITS DIFFER", flush=True)
    for v in variants:
        ms = statistics.median(times[v])
        print(f"n={n} d={d} {v:10s} median {ms:9.2f} ms  {flops / ms / 1e9:7.1f} TF/s alg  "
              f"{flops / ms / 1e9 / 1666.67:.3f} of 1667", flush=True)
    del st, x
    torch.cuda.empty_cache()
for key in ("DAL_GRAM_NC", "DAL_GRAM_NC_MIN", "DAL_GRAM_CONTIG", "DAL_GRAM_ANT"):
    os.environ.pop(key, None)
