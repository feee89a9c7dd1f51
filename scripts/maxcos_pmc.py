"""dal_max_cosine (K4) at one shape, a few launches, for rocprofv3 --pmc /
--kernel-trace.  usage: python scripts/maxcos_pmc.py NxD [m] [reps] [bf16|unit]
(unit: dal_max_cosine_unit, the folded fp16 operand)"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from dal import _lib  # noqa: E402
from dal.engine import _ptr, _stream  # noqa: E402
from dal.similarity import LabeledSet  # noqa: E402

dev = torch.device("cuda:0")
n, d = (int(v) for v in sys.argv[1].split("x"))
m = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
unit = len(sys.argv) > 4 and sys.argv[4] == "unit"
x = bench.upload(bench.host_pool(0, n, d, "uniform"), dev).to(torch.bfloat16)
L = LabeledSet(x[:m].clone(), dev)
st = torch.zeros(1, dtype=torch.int32, device=dev)
out = torch.empty(n, dtype=torch.float32, device=dev)
for _ in range(reps):
    if unit:
        _lib.call("dal_max_cosine_unit", _ptr(x), n, d, _ptr(L.unit16), L.m_pad, _ptr(out), _ptr(st), _stream(dev))
    else:
        _lib.call("dal_max_cosine", _ptr(x), n, d, _ptr(L.rows), L.m_pad, _ptr(L.inv), 0, _ptr(out), 0,
                  _ptr(st), _stream(dev))
torch.cuda.synchronize()
print("ok", n, d, m, float(out[:4].float().mean()))
