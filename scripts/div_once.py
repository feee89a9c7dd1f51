import os, sys
sys.path.insert(0, "/root/repo/distributed-active-learning_amd"); sys.path.insert(0, "/root/repo")
import torch, bench
from dal.similarity import diversity_select
cfg = bench.CONFIGS["5"]; n, d, m, k = cfg["n"], cfg["d"], cfg["m"], cfg["k"]
dev = torch.device("cuda:0")
x = bench.upload(bench.host_pool(0, n, d, cfg["dist"]), dev).to(torch.bfloat16)
lab = x[:m].clone(); cand = torch.arange(m, n, device=dev, dtype=torch.int64)
for _ in range(3):
    s = diversity_select(x, None, k, candidates=cand, device=dev, labeled_rows=lab)
torch.cuda.synchronize(); print("ok", s.indices[:3].tolist())
