"""Same-process A/B of MFMA-kernel variants with their in-kernel clock (VERDICT
r5 item 4; cdna_hip_programming.md §5.4 rule 28: what raises the held clock
for the same MFMAs is fewer bytes from beyond L2, fewer VALU and fewer LDS
bytes per MFMA).  Every library is a clock-stamped build
(scripts/variant_build.py with scripts/patches/clock_*.patch and optional
tuning constants); per round and library: WARM_S s of back-to-back launches,
then 10 launches between two HIP events, the last one stamped (clock =
d(memtime) / d(realtime) x 100 MHz, median over blocks).  Interleaved rounds,
medians reported (rule 24).  The density accumulators of every variant must
be bit-identical (exact integer accumulation).

usage: python scripts/clock_ab.py WORKLOAD NAME=LIB [NAME=LIB ...]
  WORKLOAD: gram2 | gram3 | gram:NxD[:normal] | div5"""
import os
import statistics
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dal import _lib  # noqa: E402
from clock_probe import bind, stamped  # noqa: E402

ROUNDS = int(os.environ.get("DAL_AB_ROUNDS", "3"))  # interleaved rounds per library


def main():
    w = sys.argv[1]
    libs = {}
    for spec in sys.argv[2:]:
        name, path = spec.split("=", 1)
        libs[name] = bind(path if os.path.isabs(path) else os.path.join(REPO, path))
    dev = torch.device("cuda:0")
    first = next(iter(libs.values()))
    _lib._lib = first
    if w == "div5":
        from dal.engine import _ptr, _stream
        from dal.similarity import LabeledSet

        cfg = bench.CONFIGS["5"]
        n, d, m = cfg["n"], cfg["d"], cfg["m"]
        x = bench.upload(bench.host_pool(0, n, d, cfg["dist"]), dev).to(torch.bfloat16)
        lab = bench.upload(bench.host_pool(0, m, d, cfg["dist"]), dev).to(torch.bfloat16)
        L = LabeledSet(lab, dev)
        st = torch.zeros(1, dtype=torch.int32, device=dev)
        outs = {name: torch.empty(n, dtype=torch.float32, device=dev) for name in libs}
        flops, max_blocks = 2.0 * n * m * d, 65536

        def launcher(name):
            def launch():
                _lib.call("dal_max_cosine_unit", _ptr(x), n, d, _ptr(L.unit16), L.m_pad, _ptr(outs[name]), _ptr(st),
                          _stream(dev))
            return launch

        def result(name):
            _lib._lib = libs[name]
            launcher(name)()
            return outs[name].view(torch.int32)
    else:
        from dal.engine import PoolState

        spec = {"gram2": "100000x64", "gram3": "284807x30:normal"}.get(w, w[5:])
        parts = spec.split(":")
        n, d = (int(v) for v in parts[0].split("x"))
        x = bench.upload(bench.host_pool(0, n, d, parts[1] if len(parts) > 1 else "uniform"), dev)
        pst = PoolState(x, excluded=np.arange(bench.N_EXCLUDED), device=dev)
        op = pst.gram_operand()
        accs = {name: torch.zeros(pst.n_pad, dtype=torch.int64, device=dev) for name in libs}
        flops, max_blocks = 2.0 * (n - bench.N_EXCLUDED) ** 2 * d, 16384

        def launcher(name):
            def launch():  # (accumulates: far from int64 overflow over a few thousand launches)
                pst.gram_accumulate(accs[name], op, pst.n_pad)
            return launch

        def result(name):
            _lib._lib = libs[name]
            accs[name].zero_()
            launcher(name)()
            return accs[name]
    res = {name: [] for name in libs}
    for r in range(ROUNDS):
        for name, lib in libs.items():
            _lib._lib = lib
            res[name].append(stamped(lib, launcher(name), max_blocks))
            print(f"round {r} {name}: {res[name][-1]['launch_ms']:.4f} ms", flush=True)  # (progress)
    torch.cuda.synchronize()
    ref = next(iter(libs))
    ref_out = result(ref).clone()
    for name in libs:
        same = bool(torch.equal(result(name), ref_out))
        ms = statistics.median(r["launch_ms"] for r in res[name])
        clk = statistics.median(r["clock_ghz_median"] for r in res[name])
        print({"workload": w, "lib": name, "launch_ms_median": round(ms, 4),
               "launch_ms_all": [round(r["launch_ms"], 4) for r in res[name]], "clock_ghz": round(clk, 4),
               "clock_all": [round(r["clock_ghz_median"], 4) for r in res[name]],
               "frac_of_2500": round(flops / (ms * 1e-3) / 1e12 / 2500.0, 4), "bits_equal_first": same},
              flush=True)


if __name__ == "__main__":
    main()
