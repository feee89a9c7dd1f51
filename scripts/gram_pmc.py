"""The density Gram (dal_gram_rowsum_sym + dal_gram_sym_residual) at one
shape, a few launches, for rocprofv3 --pmc / --kernel-trace (one counter
group per run).  usage: python scripts/gram_pmc.py NxD [reps] [LIB.so]
(LIB.so: an A/B build, scripts/ab_build.sh, instead of the product library)"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dal import _lib  # noqa: E402
from dal.engine import PoolState  # noqa: E402

if len(sys.argv) > 3:  # bind an A/B build in place of the product library
    import ctypes

    lib = ctypes.CDLL(os.path.abspath(sys.argv[3]))
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib._lib = lib

dev = torch.device("cuda:0")
n, d = (int(v) for v in sys.argv[1].split("x"))
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
x = bench.upload(bench.host_pool(0, n, d, "normal" if d == 30 else "uniform"), dev)
st = PoolState(x, excluded=np.arange(10), device=dev)
op = st.gram_operand()
acc = torch.zeros(st.n_pad, dtype=torch.int64, device=dev)
for _ in range(reps):
    acc.zero_()
    st.gram_accumulate(acc, op, st.n_pad)
    st.gram_residual(acc, op)
torch.cuda.synchronize()
print("ok", n, d, reps, int(acc[100]))
