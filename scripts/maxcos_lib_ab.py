"""Same-process A/B of the max-cosine kernels (K4) between two builds of
libdal.so: AB_BASE (default ab/mc_base/libdal.so) and the in-tree library.
Per shape and entry point (dal_max_cosine_unit, dal_max_cosine values-only):
outputs must be bit-identical; then back-to-back launches between two HIP
events, interleaved A/B, median of the rounds.
usage: python scripts/maxcos_lib_ab.py [NxDxM ...]"""
import ctypes
import os
import statistics
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from dal import _lib  # noqa: E402
from dal.similarity import LabeledSet  # noqa: E402

c_i64, c_p = ctypes.c_int64, ctypes.c_void_p


def bind(path):
    lib = ctypes.CDLL(path)
    lib.dal_max_cosine_unit.argtypes = [c_p, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p]
    lib.dal_max_cosine.argtypes = [c_p, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_p]
    return lib


base = bind(os.environ.get("AB_BASE", os.path.join(REPO, "ab", "mc_base", "libdal.so")))
new = bind(os.path.join(REPO, "distributed-active-learning_amd", "dal", "libdal.so"))
dev = torch.device("cuda:0")
st = torch.cuda.current_stream(dev).cuda_stream
shapes = sys.argv[1:] or ["8000000x128x1024", "8000000x64x1024", "4000000x256x1024", "2000000x128x300"]
for sh in shapes:
    n, d, m = (int(v) for v in sh.split("x"))
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand((n, d), device=dev, generator=g).to(torch.bfloat16)
    L = LabeledSet(x[:m].clone(), dev)
    s = torch.zeros(1, dtype=torch.int32, device=dev)
    outs = {}
    for kname in ("unit", "bf16"):
        for lname, lib in (("base", base), ("new", new)):
            o = torch.empty(n, dtype=torch.float32, device=dev)
            if kname == "unit":
                fn = (lambda lib=lib, o=o: lib.dal_max_cosine_unit(x.data_ptr(), n, d, L.unit16.data_ptr(), L.m_pad,
                                                                    o.data_ptr(), s.data_ptr(), st))
            else:
                fn = (lambda lib=lib, o=o: lib.dal_max_cosine(x.data_ptr(), n, d, L.rows.data_ptr(), L.m_pad,
                                                               L.inv.data_ptr(), None, o.data_ptr(), None,
                                                               s.data_ptr(), st))
            outs[(kname, lname)] = (fn, o)
    line = f"{n} x {d}, m={m}:"
    for kname in ("unit", "bf16"):
        fb, ob = outs[(kname, "base")]
        fn_, on = outs[(kname, "new")]
        assert fb() == 0 and fn_() == 0
        torch.cuda.synchronize()
        same = torch.equal(ob.view(torch.int32), on.view(torch.int32))
        t = {"base": [], "new": []}
        for _ in range(6):
            for lname, fn in (("base", fb), ("new", fn_)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                t[lname].append(e0.elapsed_time(e1) / 5)
        tb, tn = statistics.median(t["base"]), statistics.median(t["new"])
        fl = 2.0 * n * m * d
        line += (f"  {kname}: base {tb:.4f} new {tn:.4f} ms ({fl / tn / 1e9 / 2500:.3f}) "
                 f"{'bits identical' if same else 'BITS DIFFER'}")
    print(line, f"status {int(s.item())}", flush=True)
    del x, L, outs
    torch.cuda.empty_cache()
