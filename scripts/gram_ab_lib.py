"""Same-process A/B of the density Gram: the round-2 library's 3-product
symmetric kernel (ab/libdal_r02.so, built from the round-2 sources) against
the current compensated kernel (dal, libdal.so) on BASELINE shapes.  Times
prep-free density launches (the operand is prepared once per library) with
HIP events, interleaved, and checks both densities against each other within
the sum of their rigorous bounds.

usage: python scripts/gram_ab_lib.py [NxD[:normal] ...] [--reps R]
"""
import ctypes
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dal import _lib  # noqa: E402
from dal.engine import PoolState, _ptr, _stream  # noqa: E402

c_i64, c_p, c_int, c_dbl = ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_double


def old_lib():
    lib = ctypes.CDLL(os.path.join(REPO, "ab", "libdal_r02.so"))
    lib.dal_prep_split.argtypes = [c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_p]
    lib.dal_gram_rowsum_sym_skip.argtypes = [c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64,
                                             c_i64, c_p, c_int, c_p]
    lib.dal_density_error_bound_sym.restype = c_dbl
    lib.dal_density_error_bound_sym.argtypes = [c_i64]
    return lib


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 3
    shapes = args or ["100000x64", "284807x30:normal", "500000x256", "2000000x256"]
    dev = torch.device("cuda:0")
    old = old_lib()
    lib = _lib.load()
    for spec in shapes:
        dims, _, dist = spec.partition(":")
        n, d = (int(v) for v in dims.split("x"))
        dist = dist or "uniform"
        x = bench.upload(bench.host_pool(0, n, d, dist), dev)
        E = np.arange(10)
        st = PoolState(x, excluded=E, device=dev, gram="sym")
        op_new = st.gram_operand()
        nb = st.nb_active()
        # the round-2 operand (KS 64 layout at d_pad 256)
        op_old = torch.empty((st.n_pad, 2 * st.d_pad), dtype=torch.int16, device=dev)
        n64 = torch.empty(n, dtype=torch.float64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        s = _stream(dev)
        rc = old.dal_prep_split(_ptr(x), n, d, d, _ptr(st.flags), st.n_pad, st.d_pad, _ptr(op_old), _ptr(n64),
                                None, None, _ptr(status), s)
        assert rc == 0, rc
        acc_o = torch.zeros(st.n_pad, dtype=torch.int64, device=dev)
        acc_n = torch.zeros(st.n_pad, dtype=torch.int64, device=dev)
        t_old, t_new, t_res = [], [], []
        for _ in range(reps):
            for which in ("old", "new"):
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                acc = acc_o if which == "old" else acc_n
                acc.zero_()
                e0.record()
                if which == "old":
                    rc = old.dal_gram_rowsum_sym_skip(_ptr(op_old), 0, st.n_pad // 256, _ptr(op_old), 0, 0, nb, 0, 0,
                                                      nb, st.d_pad, _ptr(acc), 0, s)
                    assert rc == 0, rc
                    e1.record()
                    e2.record()
                else:
                    st.gram_accumulate(acc, op_new, st.n_pad)
                    e1.record()
                    st.gram_residual(acc, op_new)
                    e2.record()
                torch.cuda.synchronize()
                (t_old if which == "old" else t_new).append(e0.elapsed_time(e1))
                if which == "new":
                    t_res.append(e1.elapsed_time(e2))
        do = acc_o[:n].double() / 2**32
        dn = acc_n[:n].double() / 2**32
        ref = st.density_exact()
        keep = torch.ones(n, dtype=torch.bool, device=dev)
        keep[:10] = False
        bo = float(old.dal_density_error_bound_sym(n - 10))
        bn = float(lib.dal_density_error_bound_sym(n - 10))
        eo = float((do - ref)[keep].abs().max())
        en = float((dn - ref)[keep].abs().max())
        flops = 2.0 * (n - 10) * (n - 10) * d
        mo, mn, mr = np.median(t_old), np.median(t_new), np.median(t_res)
        print(f"{spec}: old {mo:.3f} ms ({flops / mo / 1e9 / 2500:.3f} of 2.5 PF) | new {mn:.3f} + residual "
              f"{mr:.3f} ms ({flops / (mn + mr) / 1e9 / 2500:.3f}) | speedup {mo / (mn + mr):.3f} | "
              f"max err old {eo:.3e} (bound {bo:.3e}) new {en:.3e} (bound {bn:.3e})", flush=True)
        if not (en <= bn and eo <= bo):
            print(f"  BOUND VIOLATED: new {en <= bn} old {eo <= bo}", flush=True)
        del x, st, op_new, op_old, acc_o, acc_n
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
