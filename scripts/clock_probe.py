"""In-kernel clock of the MFMA kernels (MI355X_MICROARCH.md 'DVFS give-back'
item 6): a timing-only build stamps s_memtime (shader
clock) and s_memrealtime (100 MHz) at each block's entry and exit
(scripts/patches/clock_*.patch through scripts/variant_build.py; the product
source carries no stamps).  After >= 2 s of back-to-back launches on the
workload's data, one more launch is stamped: clock = d(memtime) / d(realtime)
x 100 MHz per block, median / p10 / p90 over blocks; the launch's wall time
by HIP events beside it.

usage: python scripts/clock_probe.py LIB.so WORKLOAD [WORKLOAD ...]
  WORKLOAD: gram2 | gram3 | gram4 | gram:NxD[:normal]   (gram_csym_kernel, one density Gram call)
            div5                                        (maxcos_kernel<UNIT>, config 5)
LIB.so must be the matching build (ab/clock_gram or ab/clock_maxcos)."""
import ctypes
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
from dal import _lib  # noqa: E402

WARM_S = 2.5


def bind(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    lib.dal_diag_clock_read.restype = ctypes.c_int
    lib.dal_diag_clock_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.dal_diag_clock_clear.restype = ctypes.c_int
    lib.dal_diag_clock_clear.argtypes = []
    return lib


def stamped(lib, launch, max_blocks):
    """Warm for WARM_S s of back-to-back launches, then time 10 launches by
    events and stamp the last one."""
    t_end = time.perf_counter() + WARM_S
    n = 0
    while time.perf_counter() < t_end:
        for _ in range(4):
            launch()
        torch.cuda.synchronize()
        n += 4
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    assert lib.dal_diag_clock_clear() == 0
    e0.record()
    for _ in range(10):
        launch()
    e1.record()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (4 * max_blocks))()
    assert lib.dal_diag_clock_read(ctypes.addressof(buf), 4 * max_blocks) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4).astype(np.float64)
    a = a[(a[:, 1] > 0) & (a[:, 3] > a[:, 1])]
    clk = (a[:, 2] - a[:, 0]) / (a[:, 3] - a[:, 1]) * 100e6
    span_us = (a[:, 3].max() - a[:, 1].min()) / 100.0
    return dict(warm_launches=n, launch_ms=e0.elapsed_time(e1) / 10, blocks=int(a.shape[0]),
                clock_ghz_median=float(np.median(clk)) / 1e9, clock_ghz_p10=float(np.percentile(clk, 10)) / 1e9,
                clock_ghz_p90=float(np.percentile(clk, 90)) / 1e9,
                block_us_median=float(np.median(a[:, 3] - a[:, 1])) / 100.0, stamped_span_us=span_us)


def gram_workload(lib, n, d, dist):
    from dal.engine import PoolState

    _lib._lib = lib
    dev = torch.device("cuda:0")
    x = bench.upload(bench.host_pool(0, n, d, dist), dev)
    st = PoolState(x, excluded=np.arange(bench.N_EXCLUDED), device=dev)
    op = st.gram_operand()
    acc = torch.zeros(st.n_pad, dtype=torch.int64, device=dev)

    def launch():
        st.gram_accumulate(acc, op, st.n_pad)

    r = stamped(lib, launch, 16384)
    flops = 2.0 * (n - bench.N_EXCLUDED) * (n - bench.N_EXCLUDED) * d
    r["gram_tflops"] = flops / (r["launch_ms"] * 1e-3) / 1e12
    r["frac_of_2500"] = r["gram_tflops"] / 2500.0
    r["shape"] = f"{n}x{d} {dist}"
    return r


def div_workload(lib):
    from dal.engine import _ptr, _stream
    from dal.similarity import LabeledSet

    _lib._lib = lib
    cfg = bench.CONFIGS["5"]
    n, d, m = cfg["n"], cfg["d"], cfg["m"]
    dev = torch.device("cuda:0")
    x = bench.upload(bench.host_pool(0, n, d, cfg["dist"]), dev).to(torch.bfloat16)
    lab = bench.upload(bench.host_pool(0, m, d, cfg["dist"]), dev).to(torch.bfloat16)
    L = LabeledSet(lab, dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)

    def launch():
        _lib.call("dal_max_cosine_unit", _ptr(x), n, d, _ptr(L.unit16), L.m_pad, _ptr(out), _ptr(st), _stream(dev))

    r = stamped(lib, launch, 65536)
    r["tflops"] = 2.0 * n * m * d / (r["launch_ms"] * 1e-3) / 1e12
    r["frac_of_2500"] = r["tflops"] / 2500.0
    r["shape"] = f"{n}x{d} bf16 vs {m}"
    return r


def main():
    path = sys.argv[1]
    lib = bind(path if os.path.isabs(path) else os.path.join(REPO, path))
    for w in sys.argv[2:]:
        if w == "div5":
            r = div_workload(lib)
        else:
            spec = {"gram2": "100000x64", "gram3": "284807x30:normal", "gram4": "2000000x256"}.get(w, w[5:])
            parts = spec.split(":")
            n, d = (int(v) for v in parts[0].split("x"))
            r = gram_workload(lib, n, d, parts[1] if len(parts) > 1 else "uniform")
        r["workload"] = w
        print({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}, flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
