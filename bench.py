"""Benchmark: pool rows scored per second for density-weighted uncertainty
query selection (BASELINE.json metric), 1..N GPUs of one node.

One step = one cold query-selection iteration of density_weighting.py
(:58-100 proximity/density, :133-172 votes, entropy x density, top-k) over a
synthetic pool already resident in HBM: row L2-normalise -> fused fp32-MFMA
Gram row-sum (density) -> forest votes + score -> exact top-k with fp64
re-rank.  Nothing is cached across timed steps.  With N > 1 the pool is
row-sharded (strong scaling: the same pool on every N) and the two exchanges
run over RCCL.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)

METRIC = "pool rows scored/sec (density-weighted uncertainty), 1–8 GPU; % MFMA/HBM peak"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 TB/s measured float4 copy)

CONFIGS = {
    "2": dict(workload="config2: density_weighting.py cosine information density (beta=1), "
                       "synthetic U[0,1) 100,000 x 64 fp32 pool, T=10 depth-4 forest, k=100, E=L0={0..9}",
              n=100_000, d=64, trees=10, depth=4, k=100, dist="uniform"),
    "3": dict(workload="config3: credit-card shape 284,807 x 30 N(0,1) fp32, RF T=100 depth 4, "
                       "entropy x density, k=100, E={0..9}",
              n=284_807, d=30, trees=100, depth=4, k=100, dist="normal"),
    "4": dict(workload="config4: synthetic U[0,1) 2,000,000 x 256 fp32 pool, T=10 depth-4 forest, "
                       "entropy x density, k=100, E={0..9}",
              n=2_000_000, d=256, trees=10, depth=4, k=100, dist="uniform"),
    "5": dict(workload="config5: batch-mode diversity selection (similarity.py max-cosine to the labeled "
                       "set), U[0,1)->bf16 8,000,000 x 128 pool, L = first 1,024 rows, k=1000, fp32 accumulate",
              n=8_000_000, d=128, k=1000, m=1024, dist="uniform", mode="div"),
}
N_EXCLUDED = 10
GEN_CHUNK = 65536


def make_pool_rows(lo: int, hi: int, d: int, dist: str, device):
    """Rows [lo, hi) of the synthetic pool, generated on the GPU in fixed
    65,536-row chunks (seed = chunk id) so every rank/GPU count sees the same pool."""
    import torch

    out = torch.empty((hi - lo, d), dtype=torch.float32, device=device)
    c0 = lo // GEN_CHUNK
    c1 = (hi + GEN_CHUNK - 1) // GEN_CHUNK
    for c in range(c0, c1):
        g = torch.Generator(device=device)
        g.manual_seed(1_000_003 * 7 + c)
        r0, r1 = c * GEN_CHUNK, (c + 1) * GEN_CHUNK
        if dist == "uniform":
            blk = torch.rand((GEN_CHUNK, d), generator=g, device=device, dtype=torch.float32)
            blk.clamp_(min=1e-7)  # keep every row's norm > 0
        else:
            blk = torch.randn((GEN_CHUNK, d), generator=g, device=device, dtype=torch.float32)
        a, b = max(lo, r0), min(hi, r1)
        if a < b:
            out[a - lo:b - lo] = blk[a - r0:b - r0]
    return out


def cpu_baseline(x_host: np.ndarray, cfg, of, budget_s: float = 12.0):
    """Reference algorithm on the host CPU (oracle = the build's fp64 NumPy
    restatement): full fp64 Gram row-sum (BLAS matmul, as BlockMatrix.multiply)
    for a sample of rows against every column, per-tree votes, entropy LUT,
    score and the descending sort; rows/s = sample rows / elapsed."""
    from oracle import dal_oracle as O

    try:
        from threadpoolctl import threadpool_info

        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        threads = len(os.sched_getaffinity(0))
    n = x_host.shape[0]
    keep = np.ones(n, dtype=bool)
    keep[:N_EXCLUDED] = False
    U = O.l2_normalize(x_host)
    Uc = U[keep]
    ent = O.lut_entropy(cfg["trees"])

    def run(rows):
        t0 = time.perf_counter()
        sl = np.arange(N_EXCLUDED, N_EXCLUDED + rows)
        d = np.zeros(rows)
        for c0 in range(0, Uc.shape[0], 16384):
            d += (U[sl] @ Uc[c0:c0 + 16384].T).sum(axis=1)
        v = O.votes(of, x_host[sl])
        sc = ent[v] * d
        O.select_topk(sc, sl, cfg["k"], ascending=False)
        return time.perf_counter() - t0

    rows = 64
    dt = run(rows)
    rows = int(min(n - N_EXCLUDED, max(64, rows * budget_s / max(dt, 1e-3))))
    dt = run(rows)
    return {"value": rows / dt, "unit": "rows/s", "cores": int(threads), "kind": "port",
            "sample": f"{rows} pool rows scored against all {n - N_EXCLUDED} non-excluded columns "
                      f"(fp64 BLAS Gram row-sum + {cfg['trees']}-tree votes + entropy score + sort), "
                      f"{dt:.1f} s on the host"}


BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense f16 MFMA (same cycles as bf16)


def gram_roofline(gram, achieved, traffic, gram_ms, gram_ms_max, flops):
    """Roofline entry of the density GEMM.  achieved = ALGORITHMIC flops
    (2 per feature per (row, column) pair) / launch time.  The split kernel
    issues three fp16 MFMA products per algorithmic product, so its ceiling is
    the dense fp16 peak / 3; the native fp32-MFMA peak is reported beside."""
    if gram == "f32":
        return {"bound": "mfma", "kernel": "dal_gram_rowsum (v_mfma_f32_32x32x2_f32)",
                "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / FP32_MFMA_PEAK_TFLOPS, "traffic": traffic, "launch_ms": gram_ms,
                "launch_ms_max_over_ranks": gram_ms_max, "algorithmic_flops_per_launch": flops}
    if gram == "sym":
        peak = 2.0 * F16_MFMA_PEAK_TFLOPS / 3.0
        return {"bound": "mfma",
                "kernel": "dal_gram_rowsum_sym (symmetric block pairs once; 3 x v_mfma_f32_16x16x32_f16 "
                          "per 32 features: h.h, h.l, l.h)",
                "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                "peak_note": "dense fp16 MFMA peak 2500 TF/s / 3 products per algorithmic product, x2: "
                             "each block-pair product serves S_ij and S_ji (row and column sums)",
                "executed_fp16_tflops": 1.5 * achieved, "vs_fp32_mfma_peak": achieved / FP32_MFMA_PEAK_TFLOPS,
                "traffic": traffic, "launch_ms": gram_ms, "launch_ms_max_over_ranks": gram_ms_max,
                "algorithmic_flops_per_launch": flops}
    peak = F16_MFMA_PEAK_TFLOPS / 3.0
    return {"bound": "mfma",
            "kernel": "dal_gram_rowsum_split (3 x v_mfma_f32_16x16x32_f16 per 32 features: h.h, h.l, l.h)",
            "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
            "peak_note": "dense fp16 MFMA peak 2500 TF/s / 3 products per algorithmic product",
            "executed_fp16_tflops": 3.0 * achieved, "vs_fp32_mfma_peak": achieved / FP32_MFMA_PEAK_TFLOPS,
            "traffic": traffic, "launch_ms": gram_ms, "launch_ms_max_over_ranks": gram_ms_max,
            "algorithmic_flops_per_launch": flops}


def forest_roofline(n_rows, d, trees, forest_ms, config, world):
    """K2 (dal_forest_score, density mode): HBM-bound.  Algorithmic bytes per
    launch = every row's features once (n*d*4) + row flag (1) + fixed-point
    density in (8) + votes (4) + fp64 score (8) + the two interval keys (16)."""
    if not forest_ms:
        return None
    per_row = d * 4 + 1 + 8 + 4 + 8 + 16
    nbytes = float(n_rows) * per_row
    gbs = nbytes / (forest_ms * 1e-3) / 1e9
    traffic = None
    tpath = os.path.join(REPO, "profiles", "hbm_traffic.json")
    if os.path.exists(tpath) and world == 1:
        try:
            traffic = (json.load(open(tpath)).get(f"config{config}") or {}).get("forest_score_bytes_per_launch")
        except Exception:
            traffic = None
    return {"bound": "hbm", "kernel": f"dal_forest_score (T={trees} depth-4 trees, LDS-resident SoA; "
                                      "votes -> LUT -> density-weighted interval keys)",
            "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "traffic": traffic, "launch_ms": forest_ms, "algorithmic_bytes_per_launch": nbytes,
            "bytes_per_row": per_row, "note": "timed with HIP events on the launch stream over the warm "
                                              "steps (density cached, nothing concurrent)"}


def bench_diversity(args, cfg, world, rank, dev, dist, backend):
    """Config 5: one step = max-cosine of every pool row to the labeled set
    (bf16 MFMA, fp32 accumulate) + exact top-k of the least similar rows."""
    import torch

    from dal import parallel
    from dal.similarity import diversity_select

    n, d, k, m = cfg["n"], cfg["d"], cfg["k"], cfg["m"]
    lo, hi, _ = parallel.shard_range(n, world, rank)
    x = make_pool_rows(lo, hi, d, cfg["dist"], dev).to(torch.bfloat16)
    lab = make_pool_rows(0, m, d, cfg["dist"], dev).to(torch.bfloat16)
    cand = torch.arange(max(lo, m), hi, device=dev, dtype=torch.int64)
    comm = parallel.TorchComm() if world > 1 else None

    def step():
        if world > 1:
            return parallel.diversity_select_sharded(x, lo, lab, k, comm, candidates=cand, device=dev)
        s = diversity_select(x, None, k, candidates=cand, device=dev, labeled_rows=lab)
        return s.indices, s.selected_scores

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    # kernel-only timing of the max-cosine launch on this rank
    from dal import _lib
    from dal.engine import _ptr, _stream
    from dal.similarity import LabeledSet

    L = LabeledSet(lab, dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.empty(hi - lo, dtype=torch.float32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = []
    for _ in range(3):
        e0.record()
        _lib.call("dal_max_cosine", _ptr(x), hi - lo, d, _ptr(L.rows), L.m_pad, _ptr(L.inv), 0,
                  _ptr(out), _ptr(st), _stream(dev))
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    kms = sorted(ms)[1]
    tdev = dev if backend == "nccl" else "cpu"
    t = torch.tensor([elapsed, kms], dtype=torch.float64, device=tdev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0])
    flops = 2.0 * (hi - lo) * m * d
    achieved = flops / (kms * 1e-3) / 1e12
    traffic = None
    tpath = os.path.join(REPO, "profiles", "hbm_traffic.json")
    if os.path.exists(tpath) and world == 1:
        try:
            traffic = json.load(open(tpath)).get(f"config{args.config}", {}).get("maxcos_bytes_per_launch")
        except Exception:
            traffic = None
    out_line = {
        "metric": "pool rows scored/sec (diversity: max-cosine to labeled set + exact top-k)",
        "value": (n - m) * args.steps / elapsed, "unit": "rows/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed * 1000 / args.steps, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (GPU-generated, fixed seeds per 65,536-row chunk)",
        "config": {"workload": cfg["workload"], "pool_rows": n, "features": d, "labeled": m, "k": k,
                   "parallelism": f"row-shard dp{world}" if world > 1 else "single GPU"},
        "roofline": {"bound": "mfma", "kernel": "dal_max_cosine (v_mfma_f32_32x32x16_bf16)",
                     "achieved": achieved, "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / BF16_MFMA_PEAK_TFLOPS, "traffic": traffic, "launch_ms": kms,
                     "algorithmic_flops_per_launch": flops,
                     "pool_bytes_per_launch": (hi - lo) * d * 2,
                     "hbm_frac_of_8TBs": (hi - lo) * d * 2 / (kms * 1e-3) / 8e12},
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(out_line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: 50; config 4: 3)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default: 10; config 4: 1)")
    ap.add_argument("--config", default="2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--warm-steps", type=int, default=None)
    args = ap.parse_args()
    # steady-state defaults: enough steps that allocator / stream set-up of the
    # first steps is outside the timed region (a 100k-row step is ~1.5 ms)
    big = args.config == "4"
    if args.steps is None:
        args.steps = 3 if big else 50
    if args.warmup is None:
        args.warmup = 1 if big else 10
    if args.warm_steps is None:
        args.warm_steps = 3 if big else 20

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # DAL_BENCH_BACKEND=gloo rehearses the multi-process path with several
    # ranks on one GPU (all-gathers staged through the host); default: RCCL.
    backend = os.environ.get("DAL_BENCH_BACKEND", "nccl")
    n_dev = torch.cuda.device_count()
    dev = torch.device("cuda", local_rank % max(n_dev, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from dal import engine, parallel
    from dal.forest import Forest

    cfg = CONFIGS[args.config]
    if cfg.get("mode") == "div":
        return bench_diversity(args, cfg, world, rank, dev, dist, backend)
    n, d, k = cfg["n"], cfg["d"], cfg["k"]
    lo, hi, shard = parallel.shard_range(n, world, rank)
    x = make_pool_rows(lo, hi, d, cfg["dist"], dev)
    forest = Forest.synthetic(cfg["trees"], cfg["depth"], d, seed=1, dist=cfg["dist"])
    excluded = np.arange(N_EXCLUDED)
    unl = torch.arange(N_EXCLUDED, n, device=dev, dtype=torch.int64)
    n_scored = n - N_EXCLUDED

    if world > 1:
        sel = parallel.ShardedSelector(x, n, rank, world, excluded=excluded, device=dev)
        comm = parallel.TorchComm()
        state = sel.state

        def step():
            state.clear_caches()
            sel._density = None
            return parallel.select(sel, comm, unl, forest, k, mode="dw")
    else:
        state = engine.PoolState(x, excluded=excluded, device=dev)

        def step():
            state.clear_caches()
            r = engine.density_step(state, unl, forest, k)
            return r.indices, r.selected_scores

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    state.gram_events = []
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        idx, scores = step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    events = state.gram_events
    state.gram_events = None
    # the Gram launches of one step (one, or own-shard + rest when N > 1), averaged over steps
    gram_ms = sum(a.elapsed_time(b) for a, b in events) / max(args.steps, 1)
    tdev = dev if backend == "nccl" else "cpu"
    t = torch.tensor([elapsed, gram_ms], dtype=torch.float64, device=tdev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, gram_ms_max = float(t[0]), float(t[1])

    # warm path: density cached (the reference's density is constant per pool)
    warm_ms = forest_ms = None
    if args.warm_steps > 0:
        if world > 1:
            parallel.select(sel, comm, unl, forest, k, mode="dw")
        else:
            engine.density_step(state, unl, forest, k)
        torch.cuda.synchronize()
        barrier()
        state.forest_events = []
        tw = time.perf_counter()
        for _ in range(args.warm_steps):
            if world > 1:
                parallel.select(sel, comm, unl, forest, k, mode="dw")
            else:
                engine.density_step(state, unl, forest, k)
        torch.cuda.synchronize()
        barrier()
        tw = torch.tensor([time.perf_counter() - tw], dtype=torch.float64, device=tdev)
        if world > 1:
            dist.all_reduce(tw, op=dist.ReduceOp.MAX)
        warm_ms = float(tw[0]) * 1000 / args.warm_steps
        fev = state.forest_events
        state.forest_events = None
        if fev:
            forest_ms = sum(a.elapsed_time(b) for a, b in fev) / len(fev)

    # separable density mode (exact O(N*D) identity): cold step, reported beside
    sep_ms = None
    if args.warm_steps > 0:
        def sep_step():
            state.clear_caches()
            if world > 1:
                sel._density = None
                return parallel.select(sel, comm, unl, forest, k, mode="dw", density_mode="separable")
            return engine.density_step(state, unl, forest, k, mode="separable")
        sep_step()
        torch.cuda.synchronize()
        barrier()
        ts = time.perf_counter()
        for _ in range(args.warm_steps):
            sep_step()
        torch.cuda.synchronize()
        barrier()
        ts = torch.tensor([time.perf_counter() - ts], dtype=torch.float64, device=tdev)
        if world > 1:
            dist.all_reduce(ts, op=dist.ReduceOp.MAX)
        sep_ms = float(ts[0]) * 1000 / args.warm_steps

    # roofline of the dominant kernel (density Gram row-sum), this rank's launch
    rows_local = (hi - lo) - int(np.sum((excluded >= lo) & (excluded < hi)))
    flops = 2.0 * rows_local * (n - N_EXCLUDED) * d
    achieved = flops / (gram_ms * 1e-3) / 1e12 if gram_ms > 0 else 0.0
    traffic = None
    tpath = os.path.join(REPO, "profiles", "hbm_traffic.json")
    if os.path.exists(tpath):
        try:
            tr = json.load(open(tpath)).get(f"config{args.config}")
            if tr and world == 1:
                traffic = tr.get({"sym": "gram_rowsum_sym_bytes_per_launch",
                                  "split": "gram_rowsum_split_bytes_per_launch"}.get(
                                      state.gram, "gram_rowsum_bytes_per_launch"))
        except Exception:
            traffic = None

    ms_per_step = elapsed * 1000 / args.steps
    out = {
        "metric": METRIC,
        "value": n_scored * args.steps / elapsed,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32" if state.gram == "f32" else "f32 (fp16-split MFMA, fp32 accumulate)",
        "data": "synthetic (GPU-generated, fixed seeds per 65,536-row chunk); forest synthetic (seed 1)",
        "config": {"workload": cfg["workload"], "pool_rows": n, "features": d, "trees": cfg["trees"],
                   "depth": cfg["depth"], "k": k, "excluded": N_EXCLUDED, "rows_scored": n_scored,
                   "parallelism": f"row-shard dp{world} (RCCL all-gather)" if world > 1 else "single GPU"},
        "selection_latency_ms": ms_per_step,
        "warm_selection_latency_ms": warm_ms,
        "warm_rows_per_s": (n_scored / (warm_ms * 1e-3)) if warm_ms else None,
        "separable": ({"cold_selection_latency_ms": sep_ms, "rows_per_s": n_scored / (sep_ms * 1e-3),
                       "note": "density via the exact O(N*D) identity sum_j<u_i,u_j> = <u_i, sum_j u_j> "
                               "(canonical fp64, same selection); HBM-bound, not the MFMA path"}
                      if sep_ms else None),
        "roofline": gram_roofline(state.gram, achieved, traffic, gram_ms, gram_ms_max, flops),
        "roofline_forest": forest_roofline(state.n, d, cfg["trees"], forest_ms, args.config, world),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import dal_oracle as O

        of = O.synthetic_forest(cfg["trees"], cfg["depth"], d, seed=1, dist=cfg["dist"])
        out["cpu_baseline"] = cpu_baseline(x.cpu().numpy(), cfg, of)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
