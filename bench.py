"""Benchmark: pool rows scored per second for density-weighted uncertainty
query selection (BASELINE.json metric), 1..N GPUs of one node.

One step = one cold query-selection iteration of density_weighting.py
(:58-100 proximity/density, :133-172 votes, entropy x density, top-k) over a
pool already resident in HBM: row L2-normalise -> fused symmetric MFMA Gram
row-sum (density) -> forest votes + score -> exact top-k with fp64 re-rank.
Nothing is cached across timed steps.  With N > 1 the pool is row-sharded
(strong scaling: the same pool on every N) and the two all-gathers run over RCCL.

Default workload (N = 1 and N > 1): BASELINE config 4, the north-star pool
(2,000,000 x 256 U[0,1) fp32 from numpy default_rng(0), the BASELINE.md pool),
T = 10, k = 100, E = {0..9}.  Config 2 (100k x 64) runs beside it as the
``extra.config2`` key.  After timing, the bench checks its own work: the last
timed step's selection must equal (indices and fp64 scores, bit for bit) the
selection of the exact separable density path on the same pool.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py launches its
own N ranks (child processes, 127.0.0.1 rendezvous) before any GPU call and
re-prints rank 0's output, headline last; under torchrun it runs as one rank.
DAL_BENCH_SHARDED=1 with --gpus 1 runs the same step through the sharded path
(dal/parallel.py) on a one-rank RCCL group: the multi-GPU path's fixed cost at
N = 1, beside the single-GPU headline.

Output (rank 0): one compact JSON line per extra workload ({"extra": label,
...}, <= 1 KB each), then the compact headline as the LAST stdout line
(<= 4 KB: metric, value, roofline, cpu_baseline, self-checks, world size).
The full result with every note and sub-field goes to --out
(default gpurun_out/bench_full.json).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)

METRIC = "pool rows scored/sec (density-weighted uncertainty), 1–8 GPU; % MFMA/HBM peak"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 TB/s measured float4 copy)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA
# K2 / K3 launch timing: a GPU spin of this many cycles is queued ahead of each
# timed call, so its launches are submitted before the GPU reaches them and the
# HIP events bracket the device span only (not the host's submission gaps)
EVENT_LEAD_CYCLES = 2_000_000
# ... and each timed call is issued EVENT_REPEAT times between its two events
# (an event record on this stack is a marker with a cache release: several us,
# comparable to K3 itself); launch_ms = the bracket / EVENT_REPEAT
EVENT_REPEAT = 10
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense f16 MFMA (same cycles as bf16)

CONFIGS = {
    "2": dict(workload="config2: density_weighting.py cosine information density (beta=1), "
                       "U[0,1) 100,000 x 64 fp32 pool (default_rng(0)), T=10 depth-4 forest, k=100, "
                       "E=L0={0..9}",
              n=100_000, d=64, trees=10, depth=4, k=100, dist="uniform"),
    "3": dict(workload="config3: credit-card shape 284,807 x 30 N(0,1) fp32 (default_rng(0)), RF T=100 "
                       "depth 4, entropy x density, k=100, E={0..9}",
              n=284_807, d=30, trees=100, depth=4, k=100, dist="normal"),
    "4": dict(workload="config4: U[0,1) 2,000,000 x 256 fp32 pool (default_rng(0)), T=10 depth-4 forest, "
                       "entropy x density, k=100, E={0..9}",
              n=2_000_000, d=256, trees=10, depth=4, k=100, dist="uniform"),
    "5": dict(workload="config5: batch-mode diversity selection (similarity.py max-cosine to the labeled "
                       "set), U[0,1)->bf16 8,000,000 x 128 pool (default_rng(0)), L = first 1,024 rows, "
                       "k=1000, fp32 accumulate",
              n=8_000_000, d=128, k=1000, m=1024, dist="uniform", mode="div"),
}
N_EXCLUDED = 10
# DAL_BENCH_SHARDED=1: run --gpus 1 through dal/parallel.py on a one-rank
# process group (RCCL; DAL_BENCH_BACKEND=gloo for the host-staged rehearsal)
SHARDED = os.environ.get("DAL_BENCH_SHARDED", "") == "1"
# default extras beside the config-4 headline: configs 2, 3, 5
# and config 4 at T = 100 and at k = 1000
DEFAULT_EXTRA = "2,3,5,4:T100,4:k1000"


def resolve(spec: str):
    """'4', '4:T100', '4:k1000', '4:T100:k1000' -> (config key, cfg dict, label)."""
    parts = spec.split(":")
    c = parts[0]
    cfg = dict(CONFIGS[c])
    note = []
    for p in parts[1:]:
        if p[:1] == "T" and "trees" in cfg:
            cfg["trees"] = int(p[1:])
            note.append(f"T={cfg['trees']}")
        elif p[:1] == "k":
            cfg["k"] = int(p[1:])
            note.append(f"k={cfg['k']}")
        else:
            raise SystemExit(f"bad config spec {spec!r}")
    if note:
        cfg["workload"] += f" [override: {', '.join(note)}]"
    label = f"config{c}" + "".join(f"_{p}" for p in parts[1:])
    return c, cfg, label
POOL_SEED = 0
DATA_NOTE = ("synthetic: numpy default_rng(0) pool of the BASELINE.md shape (rows of a shard generated "
             "by PCG64 advance, identical for every GPU count); forest synthetic (default_rng(1))")
# K3 (dal_dw_select exact level 1) algorithmic bytes per row: the radix select
# reads the pessimistic key once per pass; the ordered compaction reads both
# interval keys twice (count, write).
TOPK_RADIX_PASSES = 6


# ------------------------------------------------------------------ pool --
def host_pool(lo: int, hi: int, d: int, dist: str, seed: int = POOL_SEED) -> np.ndarray:
    """Rows [lo, hi) of ``default_rng(seed).random((N, d), float32)`` (or
    ``standard_normal``).  Uniform rows are generated in parallel chunks, each
    from a PCG64 advanced to the chunk's first value (one 64-bit draw per two
    float32 values; chunk starts are even), so any shard is generated alone and
    equals the same rows of the full pool."""
    if dist == "normal":  # rejection sampling: not advanceable -> full pool, sliced
        return np.random.default_rng(seed).standard_normal((hi, d), dtype=np.float32)[lo:hi].copy()
    out = np.empty((hi - lo, d), dtype=np.float32)
    chunk = 65536

    def fill(r0):
        r1 = min(r0 + chunk, hi)
        g = np.random.default_rng(seed)
        g.bit_generator.advance(r0 * d // 2)
        out[r0 - lo:r1 - lo] = g.random((r1 - r0, d), dtype=np.float32)

    starts = list(range(lo, hi, chunk))
    if starts and (lo * d) % 2:
        raise ValueError("shard start must be an even value offset")
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        list(ex.map(fill, starts))
    return out


def upload(x: np.ndarray, dev):
    import torch

    return torch.from_numpy(x).to(dev)


# ------------------------------------------------------------ baselines --
def _cores():
    try:
        from threadpoolctl import threadpool_info

        return max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        return len(os.sched_getaffinity(0))


def cpu_baseline(x_host: np.ndarray, cfg, of, budget_s: float = 12.0):
    """Reference algorithm on the host CPU (oracle = the build's fp64 NumPy
    restatement): full fp64 Gram row-sum (BLAS matmul, as BlockMatrix.multiply)
    for a sample of rows against every column, per-tree votes, entropy LUT,
    score and the descending sort; rows/s = sample rows / elapsed."""
    from oracle import dal_oracle as O

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

    def run_sep(rows):
        # variant (ii) of SURVEY §8(d): the separable fp64 density on a leading
        # slice taken as the whole pool (normalise, column sum, one dot per row)
        t0 = time.perf_counter()
        xs = x_host[:rows]
        us = O.l2_normalize(xs)[N_EXCLUDED:]
        d = us @ us.sum(axis=0)
        v = O.votes(of, xs[N_EXCLUDED:])
        O.select_topk(ent[v] * d, np.arange(N_EXCLUDED, rows), cfg["k"], ascending=False)
        return time.perf_counter() - t0

    rows = 64
    dt = run(rows)
    rows = int(min(n - N_EXCLUDED, max(64, rows * budget_s / max(dt, 1e-3))))
    dt = run(rows)
    full = rows >= n - N_EXCLUDED
    srows = min(n, 65536)
    sdt = run_sep(srows)
    srows = int(min(n, max(srows, srows * (budget_s / 3) / max(sdt, 1e-3))))
    sdt = run_sep(srows)
    sep = {"value": (srows - N_EXCLUDED) / sdt, "unit": "rows/s",
           "sample": f"first {srows} pool rows as the pool: fp64 normalise + column sum + one dot per row "
                     f"+ votes + score + sort, {sdt:.1f} s"}
    return {"value": rows / dt, "unit": "rows/s", "cores": int(_cores()), "kind": "port", "separable": sep,
            "sample": f"{rows} pool rows scored against all {n - N_EXCLUDED} non-excluded columns "
                      f"(fp64 BLAS Gram row-sum + {cfg['trees']}-tree votes + entropy score + sort), "
                      f"{dt:.1f} s on the host" + ("" if full else "; rows/s of the sample (the O(N^2) "
                                                    "per-row cost is the same for every row)")}


def cpu_baseline_div(x_host_bf16_as_f32: np.ndarray, m: int, k: int, n_total: int, budget_s: float = 12.0):
    """Config 5 on the host: fp64 max-cosine of a row slice to the labeled set
    (BLAS) + the k smallest; rows/s of the slice (the per-row cost is constant,
    so the full 8M-row job time is the slice rate extrapolated linearly)."""
    from oracle import dal_oracle as O

    lab = O.l2_normalize(x_host_bf16_as_f32[:m])

    def run(rows):
        t0 = time.perf_counter()
        U = O.l2_normalize(x_host_bf16_as_f32[m:m + rows])
        mx = (U @ lab.T).max(axis=1)
        O.select_topk(mx, np.arange(m, m + rows), k, ascending=True)
        return time.perf_counter() - t0

    rows = 4096
    dt = run(rows)
    rows = int(min(x_host_bf16_as_f32.shape[0] - m, max(4096, rows * budget_s / max(dt, 1e-3))))
    dt = run(rows)
    return {"value": rows / dt, "unit": "rows/s", "cores": int(_cores()), "kind": "port",
            "sample": f"{rows}-row slice (of {n_total - m}) scored against the {m} labeled "
                      f"rows (fp64 BLAS max-cosine + top-{k}), {dt:.1f} s on the host; linear "
                      f"extrapolation to the full pool = {(n_total - m) / (rows / dt):.0f} s"}


# ------------------------------------------------------------ rooflines --
def gram_roofline(gram, achieved, traffic, gram_ms, gram_ms_max, flops, products=3):
    """Roofline entry of the density GEMM.  achieved = ALGORITHMIC flops
    (2 per feature per (row, column) pair, every pair of the N x N Gram) /
    launch time; frac = achieved / the dense fp16 MFMA peak (2.5 PF) the
    kernel issues on.  The symmetric kernel multiplies each block pair once
    (S_ij and S_ji from one product) with ``products`` fp16 MFMA products per
    feature pair, so it executes products / 2 fp16 flops per algorithmic
    flop: ``mfma_util_executed`` is that executed rate over the same peak."""
    if gram == "f32":
        return {"bound": "mfma", "kernel": "dal_gram_rowsum (v_mfma_f32_32x32x2_f32)",
                "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / FP32_MFMA_PEAK_TFLOPS, "traffic": traffic, "launch_ms": gram_ms,
                "launch_ms_max_over_ranks": gram_ms_max, "algorithmic_flops_per_launch": flops}
    sym = gram == "sym"
    executed = achieved * products / (2.0 if sym else 1.0)
    names = {3: "h.h, h.l, l.h", 2: "H.H, H.L on the taker side + the exact closed-form remainder "
                                     "(dal_gram_sym_residual, included in launch_ms); column sums from "
                                     "sigma_P MFMAs (+3 % executed, not counted in achieved)"}
    return {"bound": "mfma",
            "kernel": (f"dal_gram_rowsum_{'sym + dal_gram_sym_residual' if sym else 'split'} "
                       f"({products}x v_mfma_f32_16x16x32_f16 / 32 features)"),
            "kernel_note": (f"{'symmetric block pairs once; ' if sym else ''}{products} fp16 products per 32 "
                            f"features: {names.get(products, '')}"),
            "achieved": achieved, "peak": F16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / F16_MFMA_PEAK_TFLOPS,
            "peak_note": "dense fp16 MFMA peak (MI355X_MICROARCH.md); achieved counts the algorithmic "
                         "2*N_rows*(N-|E|)*D flops of the full Gram",
            "executed_fp16_tflops": executed, "mfma_util_executed": executed / F16_MFMA_PEAK_TFLOPS,
            "fp16_products_per_feature_pair": products, "symmetric_pairs": sym,
            "vs_fp32_mfma_peak": achieved / FP32_MFMA_PEAK_TFLOPS,
            "traffic": traffic, "launch_ms": gram_ms, "launch_ms_max_over_ranks": gram_ms_max,
            "algorithmic_flops_per_launch": flops}


def _traffic(config, key, world):
    tpath = os.path.join(REPO, "profiles", "hbm_traffic.json")
    if world != 1 or not os.path.exists(tpath):
        return None
    try:
        return (json.load(open(tpath)).get(f"config{config}") or {}).get(key)
    except Exception:
        return None


def forest_roofline(n_rows, d, trees, forest_ms, config, world, used_features=None):
    """K2 (dal_forest_score, density mode).  Algorithmic bytes per launch =
    every row's features once (n*d*4) + row flag (1) + fixed-point density in
    (8) + votes (4) + fp64 score (8) + the two interval keys (16).  At T = 10
    the kernel streams HBM; at T = 100 (config 3) the LDS traversal (4 levels
    x T trees per row: a node read + a feature gather per level) and its
    instruction issue bound it, so the HBM fraction is reported with bound
    "lds-issue" (counters: profiles/r02/forest_config3_pmc.csv).
    used_features: the warm steps ran the blocked kernel (ABI v9,
    dal_forest_score_blocked), which reads only the forest's distinct tested
    features: those count instead of d (the row-major kernel's bytes are
    reported beside)."""
    if not forest_ms:
        return None
    tail = 1 + 8 + 4 + 8 + 16
    feats = d if used_features is None else used_features
    per_row = feats * 4 + tail
    nbytes = float(n_rows) * per_row
    gbs = nbytes / (forest_ms * 1e-3) / 1e9
    kernel = (f"dal_forest_score (T={trees} depth-4 trees, LDS-resident SoA; "
              "votes -> LUT -> density-weighted interval keys)")
    if used_features is not None:
        kernel = (f"dal_forest_score_blocked (T={trees} depth-4 trees over the pool's blocked feature-major copy: "
                  f"the {used_features} of {d} features the forest tests, 256-B runs per 64-row tile by LDS-DMA; "
                  "votes -> LUT -> density-weighted interval keys)")
    out = {"bound": "hbm" if trees <= 32 else "lds-issue",
           "kernel": kernel,
           "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
           "traffic": _traffic(config, "forest_blocked_bytes_per_launch" if used_features is not None
                               else "forest_score_bytes_per_launch", world), "launch_ms": forest_ms,
           "algorithmic_bytes_per_launch": nbytes, "bytes_per_row": per_row,
           "note": "timed with HIP events on the launch stream over the warm steps (density cached), each call queued behind a GPU spin and issued 10x back to back between the events (device time per call incl. its launch gaps; no host submission gaps, event cost amortised)"}
    if trees > 32 and used_features is None:
        out["counters"] = ("PMC per launch at config 3 (profiles/r02/forest_config3_pmc.csv): LDS array busy "
                           "SQ_LDS_IDX_ACTIVE, 42% of it bank-conflict cycles (lane-divergent feature gathers); "
                           "waves parked on s_waitcnt 51% / issue-stalled 22% / issuing 27% of their cycles")
    elif trees > 32:
        out["counters"] = ("the blocked kernel's gathers are conflict-free (rows on lanes, feature-major tile); "
                           "at T > 32 its 4 x T dependent node-then-feature LDS visits per row bound it, not HBM")
    if used_features is not None:
        out["used_features"] = used_features
        out["row_major_bytes_per_row"] = d * 4 + tail
    return out


def topk_roofline(n_rows, select_ms, config, world, level1_passes=0, step_select_ms=None):
    """K3 (dal_dw_select).  Exact level 1: radix select of the k-th
    pessimistic key (6 passes x 8 B per row) + ordered compaction (count and
    write: both interval keys, 2 x 16 B per row).  Fast level 1 (the engine
    default on pools whose candidates fit 4,096 slots): both interval keys read
    once for the row-group minima (16 B per row); the threshold, the scan of
    the groups that can hold candidates, the exact fp64 re-rank and the
    one-block sort touch O(groups + candidates) bytes.

    ``step_select_ms`` (one GPU, fast level 1): the selection launch of the
    fused step alone -- what dal_dw_step and the warm plan run after the score
    kernel has folded the row-group minima (DAL_STEP_SELECT_ONLY calls).  Its
    bytes are O(groups + candidates), so it is reported as latency-bound
    (``fused_step_select_ms``); ``launch_ms`` / ``frac`` stay the standalone
    dal_dw_select call with its own minima pass."""
    if not select_ms:
        return None
    if level1_passes:
        per_row = 16
        kernel = ("dal_dw_select (fast level 1: row-group minima -> tau = k-th group minimum -> candidate append "
                  "with in-place fp64 re-rank -> last-block sort; 2 launches)")
    else:
        per_row = 8 * TOPK_RADIX_PASSES + 32
        kernel = "dal_dw_select (radix select + interval compaction + fp64 re-rank + sort)"
    nbytes = float(n_rows) * per_row
    gbs = nbytes / (select_ms * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": kernel,
            "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "traffic": _traffic(config, "dw_select_bytes_per_launch", world), "launch_ms": select_ms,
            "fused_step_select_ms": step_select_ms,
            "fused_step_select_note": ("summary_select_kernel as dal_dw_step / the warm plan run it (row-group "
                                       "minima folded by the score kernel), timed alone: DAL_STEP_SELECT_ONLY "
                                       "calls, 10 per event pair behind a GPU spin; latency-bound. The repeats "
                                       "find the candidate rows cache-warm: in the warm plan's kernel trace, "
                                       "right after the score kernel, the same launch took 23.7 us at config 4 "
                                       "(profiles/r05/warm/timeline_config4_warm.txt)"),
            "algorithmic_bytes_per_launch": nbytes, "bytes_per_row": per_row,
            "note": "one C-ABI call (all its launches), HIP events on the launch stream, warm steps, each call queued behind a GPU spin and issued 10x back to back between the events (device time per call incl. its launch gaps; no host submission gaps, event cost amortised)"}


# ----------------------------------------------------------- workloads --
def _timed(fn, steps, barrier):
    import torch

    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize()
    barrier()
    return time.perf_counter() - t0, out


def _max_over_ranks(vals, world, dist, tdev):
    import torch

    t = torch.tensor(vals, dtype=torch.float64, device=tdev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t]


def host_colsum64(x_host: np.ndarray, lo: int, n_excluded: int, chunk: int = 65536) -> np.ndarray:
    """fp64 sum of the unit rows u_j = x_j / ||x_j|| of this rank's rows that
    are not in E = {0..n_excluded-1} (global indices; rows [lo, lo + len)).
    numpy, independent of the library: the reference for the accuracy block."""
    n_loc, d = x_host.shape
    s = np.zeros(d, dtype=np.float64)
    for c0 in range(0, n_loc, chunk):
        xc = x_host[c0:c0 + chunk].astype(np.float64)
        xc /= np.sqrt(np.einsum("ij,ij->i", xc, xc))[:, None]
        xc[np.arange(lo + c0, lo + c0 + xc.shape[0]) < n_excluded] = 0.0
        s += xc.sum(axis=0)
    return s


def sample_rows(n_loc: int, lo: int, n_excluded: int, m: int) -> np.ndarray:
    """Up to m evenly spaced local rows outside E (always the shard's first and last scored rows)."""
    first = max(0, n_excluded - lo)
    if first >= n_loc:
        return np.zeros(0, dtype=np.int64)
    return np.unique(np.linspace(first, n_loc - 1, min(m, n_loc - first)).round().astype(np.int64))


def density_accuracy(x_host, lo, gram_density, colsum, n_excluded, m=4096):
    """SURVEY §8(d) accuracy instrumentation: the Gram-path density of m
    sampled rows against d_i = <u_i, s> in fp64 on the host (``colsum`` = s
    over every row outside E).  Returns (max, mean) relative error and the
    smallest |d_ref| of the sample, the max absolute error, and the sample size."""
    pick = sample_rows(x_host.shape[0], lo, n_excluded, m)
    if pick.size == 0:
        return 0.0, 0.0, float("inf"), 0.0, 0
    xs = x_host[pick].astype(np.float64)
    xs /= np.sqrt(np.einsum("ij,ij->i", xs, xs))[:, None]
    d_ref = xs @ colsum
    err = np.abs(np.asarray(gram_density(pick), dtype=np.float64) - d_ref)
    rel = err / np.abs(d_ref)
    return float(rel.max()), float(rel.mean()), float(np.abs(d_ref).min()), float(err.max()), int(pick.size)


def abs_rowsum_tolerance(x_host, pick, gram_density, n_excluded, m=256, chunk=32768):
    """SURVEY §8(d) config-3 tolerance form: max_i |d_gram_i - d_ref_i| / sum_j |S_ij|
    (j outside E) over m of the sampled rows, fp64 on the host over every
    column (one GPU: the host holds the whole pool)."""
    pick = pick[np.linspace(0, pick.size - 1, min(m, pick.size)).round().astype(np.int64)]
    us = x_host[pick].astype(np.float64)
    us /= np.sqrt(np.einsum("ij,ij->i", us, us))[:, None]
    d_ref = np.zeros(pick.size)
    a_ref = np.zeros(pick.size)
    for c0 in range(max(n_excluded, 0), x_host.shape[0], chunk):
        xc = x_host[c0:c0 + chunk].astype(np.float64)
        xc /= np.sqrt(np.einsum("ij,ij->i", xc, xc))[:, None]
        S = us @ xc.T
        d_ref += S.sum(axis=1)
        a_ref += np.abs(S).sum(axis=1)
    err = np.abs(np.asarray(gram_density(pick), dtype=np.float64) - d_ref)
    return float((err / a_ref).max())


_POOLS = {}


def cached_pool(n, d, dist, lo, hi, dev):
    """(host rows [lo, hi), device copy) of a BASELINE pool, generated once per
    process (the config-4 variants share the 2M x 256 pool)."""
    key = (n, d, dist, lo, hi)
    if key not in _POOLS:
        _POOLS.clear()  # keep one pool resident
        x_host = host_pool(lo, hi, d, dist)
        _POOLS[key] = (x_host, upload(x_host, dev))
    return _POOLS[key]


def time_step_select(state, forest, flags, dens, lut_dev, k: int, beta: float, xb=None):
    """PoolState.step_select_probe: the selection launch of the fused step
    (what dal_dw_step and the warm plan run after the score kernel folded the
    row-group minima) timed on its own.  One full dal_dw_step keeps the minima
    (DAL_STEP_KEEP_GROUPS), then EVENT_REPEAT DAL_STEP_SELECT_ONLY calls run
    between two events (behind a GPU spin), then one more clears them.  The
    selections must equal the step's; the events go to state.step_select_events."""
    import torch

    from dal import _lib
    from dal._lib import DAL_STEP_KEEP_GROUPS, DAL_STEP_SELECT_ONLY, DAL_STEP_WS_CLEAN, call
    from dal.engine import _fprep, _ptr, _stream, candidate_cap, density_error, level1_passes, workspace

    lib = _lib.load()
    n, dev = state.n, state.device
    inner, leaf = forest.device(dev)
    norm64, colsum = state.norms(), state.colsum()
    base = candidate_cap(n, k) if state.cap_base is None else max(int(k), int(state.cap_base))
    cap = int(min(n, base * state.cap_scale))
    passes = level1_passes(state, n, k, cap)
    if passes == 0:
        return
    wsb = int(lib.dal_dw_step_workspace_bytes(n, k, cap))
    ws, wsp = workspace(wsb, dev)
    ws.zero_()
    bufs = [torch.empty(n, dtype=t, device=dev) for t in (torch.int32, torch.float64, torch.int64, torch.int64)]
    outs = [(torch.empty(k, dtype=torch.int64, device=dev), torch.empty(k, dtype=torch.float64, device=dev))
            for _ in range(2)]
    status = torch.zeros(1, dtype=torch.int32, device=dev)

    def step(flags_bits, out):
        call("dal_dw_step", _ptr(state.x), 0 if xb is None else _ptr(xb), _fprep(forest, state, xb), n, state.d,
             state.d, _ptr(inner),
             _ptr(leaf), forest.n_trees, forest.depth, _ptr(lut_dev), _ptr(dens), float(density_error(state)),
             _ptr(flags), float(beta),
             state.row_base, _ptr(norm64), _ptr(colsum), k, cap, passes, flags_bits, wsp, wsb,
             *[_ptr(b) for b in bufs], _ptr(out[0]), _ptr(out[1]), 0, _ptr(status), 0, _stream(dev))

    step(DAL_STEP_WS_CLEAN | DAL_STEP_KEEP_GROUPS, outs[0])
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    if state.event_lead_cycles:
        torch.cuda._sleep(state.event_lead_cycles)
    ev[0].record()
    for _ in range(state.event_repeat):
        step(DAL_STEP_WS_CLEAN | DAL_STEP_KEEP_GROUPS | DAL_STEP_SELECT_ONLY, outs[1])
    ev[1].record()
    step(DAL_STEP_WS_CLEAN | DAL_STEP_SELECT_ONLY, outs[1])  # the last one clears the minima
    if int(status.item()) != 0 or not (torch.equal(outs[0][0], outs[1][0]) and
                                      torch.equal(outs[0][1].view(torch.int64), outs[1][1].view(torch.int64))):
        return  # (an overflow or a mismatch: no timing recorded)
    state.step_select_events.append(ev)


def bench_dw(args, config, steps, warmup, warm_steps, world, rank, dev, dist, backend, cpu=True, cfg=None):
    """Density-weighted selection on one config; returns the JSON dict.

    The step runs through the sharded path (dal/parallel.py) when world > 1,
    or at world 1 when DAL_BENCH_SHARDED=1 (an RCCL group of one rank: the
    multi-GPU path's fixed cost on record beside the single-GPU headline)."""
    import torch

    from dal import engine, parallel
    from dal.forest import Forest

    cfg = CONFIGS[config] if cfg is None else cfg
    n, d, k = cfg["n"], cfg["d"], cfg["k"]
    lo, hi, _ = parallel.shard_range(n, world, rank)
    x_host, x = cached_pool(n, d, cfg["dist"], lo, hi, dev)  # this rank's rows (world 1: the whole pool)
    forest = Forest.synthetic(cfg["trees"], cfg["depth"], d, seed=1, dist=cfg["dist"])
    excluded = np.arange(N_EXCLUDED)
    unl = torch.arange(N_EXCLUDED, n, device=dev, dtype=torch.int64)
    n_scored = n - N_EXCLUDED
    tdev = dev if backend == "nccl" else "cpu"

    sharded = world > 1 or SHARDED

    def barrier():
        if world > 1:
            dist.barrier()

    if sharded:
        sel = parallel.ShardedSelector(x, n, rank, world, excluded=excluded, device=dev)
        comm = parallel.TorchComm()
        state = sel.state

        def step(density_mode="gram", cold=True):
            if cold:
                sel.clear_caches()
            return parallel.select(sel, comm, unl, forest, k, mode="dw", density_mode=density_mode)
    else:
        state = engine.PoolState(x, excluded=excluded, device=dev)

        def step(density_mode="gram", cold=True):
            if cold:
                state.clear_caches()
            r = engine.density_step(state, unl, forest, k, mode=density_mode)
            return r.indices, r.selected_scores

    for _ in range(warmup):
        step()
    state.gram_events, state.residual_events = [], []
    if sharded:
        sel.exchange_events = []
    elapsed, (idx_g, sc_g) = _timed(step, steps, barrier)
    events, state.gram_events = state.gram_events, None
    res_events, state.residual_events = state.residual_events, []
    # the density launches of one step (the Gram: one, or own-shard + rest when
    # N > 1; plus the compensation's closed-form remainder), averaged over steps
    resid_ms = sum(a.elapsed_time(b) for a, b in res_events) / max(steps, 1)
    gram_ms = sum(a.elapsed_time(b) for a, b in events) / max(steps, 1) + resid_ms
    ranks = None
    if sharded:  # the density exchange's collectives, per step, and their max over ranks
        xev, sel.exchange_events = sel.exchange_events, None
        ag_ms = sum(a.elapsed_time(b) for nm, a, b in xev if nm == "all_gather") / max(steps, 1)
        gram_min = -_max_over_ranks([-gram_ms], world, dist, tdev)[0]
        g_max, ag_max = _max_over_ranks([gram_ms, ag_ms], world, dist, tdev)
        ranks = {"gram_ms_max": g_max, "gram_ms_min": gram_min, "all_gather_ms_max": ag_max}
    elapsed, gram_ms_max = _max_over_ranks([elapsed, gram_ms], world, dist, tdev)

    # accuracy (outside the timed region): the timed step's
    # Gram density on sampled rows vs an fp64 host restatement
    s_host = host_colsum64(x_host, lo, N_EXCLUDED)
    if world > 1:
        t = torch.from_numpy(s_host).to(tdev)
        dist.all_reduce(t)
        s_host = t.cpu().numpy()
    dens_gram = state.density("gram")
    acc_max, acc_mean, dref_min, abs_max, n_acc = density_accuracy(
        x_host, lo, lambda pick: dens_gram[torch.from_numpy(pick).to(dev)].cpu().numpy(), s_host, N_EXCLUDED)
    tol_abs = None
    if world == 1 and cfg["dist"] == "normal" and n * d <= 20_000_000:  # signed data (config 3)
        tol_abs = abs_rowsum_tolerance(x_host, sample_rows(n, 0, N_EXCLUDED, 4096),
                                       lambda pick: dens_gram[torch.from_numpy(pick).to(dev)].cpu().numpy(),
                                       N_EXCLUDED)
    del dens_gram
    err_bound = float(engine.density_error(state))
    n_cols = n - N_EXCLUDED
    acc_max, acc_mean_max, bound_rel, abs_ncols = _max_over_ranks(
        [acc_max, acc_mean, err_bound / dref_min, abs_max / n_cols], world, dist, tdev)

    # self-check (outside the timed region): the timed step's selection equals
    # the exact separable-density selection, indices and fp64 score bits
    idx_s, sc_s = step("separable")
    same = bool(torch.equal(idx_g, idx_s)) and bool(torch.equal(sc_g.view(torch.int64), sc_s.view(torch.int64)))
    if not same:
        raise SystemExit(f"bench self-check FAILED: gram-mode selection != separable-mode selection "
                         f"({idx_g[:8].tolist()} vs {idx_s[:8].tolist()})")

    # warm path: density cached (the reference's density is constant per pool)
    warm_ms = forest_ms = select_ms = step_select_ms = forest_used = None
    warm_same = None
    if warm_steps > 0:
        step()
        # per-kernel HIP-event timing of K2 / K3 (eager launches, events on the launch stream)
        state.forest_events, state.select_events = [], []
        state.step_select_events = [] if not sharded else None
        state.step_select_probe = time_step_select if not sharded else None
        state.event_lead_cycles, state.event_repeat = EVENT_LEAD_CYCLES, EVENT_REPEAT
        for _ in range(min(warm_steps, 20)):
            step(cold=False)
        torch.cuda.synchronize()
        fev, sev, ssev = state.forest_events, state.select_events, state.step_select_events
        state.forest_events = state.select_events = state.step_select_events = state.step_select_probe = None
        state.event_lead_cycles, state.event_repeat = 0, 1
        if fev:
            forest_ms = sum(a.elapsed_time(b) for a, b in fev) / len(fev) / EVENT_REPEAT
            # the warm steps' K2 read the blocked copy: the forest's distinct tested features
            if state._xb is not None:
                forest_used = int(np.unique(forest.inner[..., 0]).size)
        if sev:
            select_ms = sum(a.elapsed_time(b) for a, b in sev) / len(sev) / EVENT_REPEAT
        if ssev:
            step_select_ms = sum(a.elapsed_time(b) for a, b in ssev) / len(ssev) / EVENT_REPEAT
        # warm latency: the step as a user runs it (one GPU: the hipGraph replay)
        step(cold=False)
        tw, (idx_w, sc_w) = _timed(lambda: step(cold=False), warm_steps, barrier)
        (tw,) = _max_over_ranks([tw], world, dist, tdev)
        warm_ms = tw * 1000 / warm_steps
        warm_same = bool(torch.equal(idx_w, idx_g)) and bool(torch.equal(sc_w.view(torch.int64),
                                                                          sc_g.view(torch.int64)))
        if not warm_same:
            raise SystemExit("bench self-check FAILED: warm-step selection != cold-step selection")

    # separable density mode (exact O(N*D) identity): cold step, reported beside
    sep_ms = None
    if warm_steps > 0:
        step("separable")
        ts, _ = _timed(lambda: step("separable"), warm_steps, barrier)
        (ts,) = _max_over_ranks([ts], world, dist, tdev)
        sep_ms = ts * 1000 / warm_steps

    # k-th boundary gap: the (k+1)-best score from the exact path, beside the
    # observed Gram error (the exact re-rank makes the selection independent of it)
    if sharded:
        _, sc_k1 = parallel.select(sel, comm, unl, forest, k + 1, mode="dw", density_mode="separable")
    else:
        sc_k1 = engine.density_step(state, unl, forest, k + 1, mode="separable").selected_scores
    sk = sc_k1.cpu().numpy()
    gap_rel = float((sk[k - 1] - sk[k]) / abs(sk[k - 1])) if len(sk) > k and sk[k - 1] != 0 else None

    # roofline of the dominant kernel (density Gram row-sum), this rank's launch
    rows_local = (hi - lo) - int(np.sum((excluded >= lo) & (excluded < hi)))
    flops = 2.0 * rows_local * (n - N_EXCLUDED) * d
    achieved = flops / (gram_ms * 1e-3) / 1e12 if gram_ms > 0 else 0.0
    traffic = _traffic(config, "gram_csym_bytes_per_launch" if state.gram == "sym"
                       else "gram_rowsum_bytes_per_launch", world)
    ms_per_step = elapsed * 1000 / steps
    out = {
        "metric": METRIC,
        "value": n_scored * steps / elapsed,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32" if state.gram == "f32" else "f32 (fp16-split MFMA, fp32 accumulate)",
        "data": DATA_NOTE,
        "config": {"workload": cfg["workload"], "pool_rows": n, "features": d, "trees": cfg["trees"],
                   "depth": cfg["depth"], "k": k, "excluded": N_EXCLUDED, "rows_scored": n_scored,
                   "parallelism": (f"row-shard dp{world} ({'RCCL' if backend == 'nccl' else backend} all-gather)"
                                   if sharded else "single GPU")},
        "selection_latency_ms": ms_per_step,
        "warm_selection_latency_ms": warm_ms,
        "warm_path": ("hipGraph replay (votes/score + row-group minima -> candidate search -> fp64 re-rank -> "
                      "sort) + input refresh, one status read" if not sharded and state.use_graphs
                      else "per-rank dal_dw_plan replay -> packed all-gather -> one-launch merge, one status read"
                      if sharded and state.use_graphs else "eager launches"),
        "warm_rows_per_s": (n_scored / (warm_ms * 1e-3)) if warm_ms else None,
        "self_check": {"gram_selection_equals_separable_selection": same,
                       "warm_selection_equals_cold_selection": warm_same, "k": k,
                       "note": "last timed step vs the exact O(N*D) density path, and the last warm step "
                               "vs the cold one: indices + fp64 score bits"},
        "accuracy": {"density_max_rel_err": acc_max, "density_mean_rel_err": acc_mean_max,
                     "density_max_abs_err_over_ncols": abs_ncols,
                     "density_err_bound_over_ncols": err_bound / n_cols,
                     "density_max_err_over_abs_rowsum": tol_abs,
                     "sampled_rows_per_rank": n_acc,
                     "density_err_bound_rel": bound_rel,
                     "kth_gap_rel": gap_rel,
                     "note": "Gram-path density (MFMA, fixed point) of evenly spaced sampled rows vs "
                             "<u_i, sum_j u_j> in fp64 numpy on the host (max over ranks); *_over_ncols: "
                             "absolute errors / (N - |E|) >= sum_j |S_ij| / (N - |E|) scale, the form "
                             "for signed data; *_over_abs_rowsum: |dd_i| / sum_j |S_ij| on 256 of the "
                             "sampled rows (SURVEY config-3 tolerance 1e-5; signed one-GPU pools); "
                             "the bound is the rigorous interval "
                             "half-width; "
                             "kth_gap_rel = (s_k - s_k+1) / |s_k| of the exact scores (the selection "
                             "itself is exact: interval keys + fp64 re-rank)"},
        "separable": ({"cold_selection_latency_ms": sep_ms, "rows_per_s": n_scored / (sep_ms * 1e-3),
                       "note": "density via the exact O(N*D) identity sum_j<u_i,u_j> = <u_i, sum_j u_j> "
                               "(canonical fp64, same selection); HBM-bound, not the MFMA path"}
                      if sep_ms else None),
        "roofline": dict(gram_roofline(state.gram, achieved, traffic, gram_ms, gram_ms_max, flops,
                                       engine.gram_products(state)), residual_ms=resid_ms),
        "roofline_forest": forest_roofline(state.n, d, cfg["trees"], forest_ms, config, world,
                                           used_features=forest_used),
        "roofline_topk": topk_roofline(state.n, select_ms, config, world,
                                       engine.LEVEL1_PASSES if state.level1_fast else 0, step_select_ms),
        "cpu_baseline": None,
        "ranks": ranks,
    }
    if rank == 0 and world == 1 and cpu and not args.no_cpu_baseline:
        from oracle import dal_oracle as O

        of = O.synthetic_forest(cfg["trees"], cfg["depth"], d, seed=1, dist=cfg["dist"])
        out["cpu_baseline"] = cpu_baseline(x_host, cfg, of, budget_s=cpu if isinstance(cpu, float) else 12.0)
    del state, x
    if sharded:
        del sel
    torch.cuda.empty_cache()
    return out


def canon_unit(x64: np.ndarray) -> np.ndarray:
    """u = x / ||x|| with ||x||^2 summed sequentially over features (mul, then
    add), as the library's canonical fp64 re-rank (numpy; no library code)."""
    n2 = np.zeros(x64.shape[0])
    for f in range(x64.shape[1]):
        n2 = n2 + x64[:, f] * x64[:, f]
    return x64 / np.sqrt(n2)[:, None]


def canon_maxcos(rows64: np.ndarray, lab64: np.ndarray) -> np.ndarray:
    """Canonical fp64 max-cosine of rows to the labeled rows: cos summed
    sequentially over features, max over the labeled set."""
    u, ul = canon_unit(rows64), canon_unit(lab64)
    S = np.zeros((u.shape[0], ul.shape[0]))
    for f in range(u.shape[1]):
        S = S + u[:, f, None] * ul[None, :, f]
    return S.max(axis=1)


def div_self_check(x_dev, lab_host64, lo, m, idx, sc, k, n_sample=4096):
    """Config-5 selection checked on the host (outside the timed region): the
    selected scores are the canonical fp64 max-cos of the selected rows, bit
    for bit; no sampled candidate row outside the selection beats the k-th
    selected score (ties by index)."""
    import torch

    idx_h = idx.cpu().numpy()
    sc_h = sc.cpu().numpy()
    rows = x_dev[torch.from_numpy(idx_h - lo).to(x_dev.device)].float().cpu().numpy().astype(np.float64)
    exact = bool(np.array_equal(canon_maxcos(rows, lab_host64).view(np.int64), sc_h.view(np.int64)))
    sorted_ok = bool(np.all((sc_h[1:] > sc_h[:-1]) | ((sc_h[1:] == sc_h[:-1]) & (idx_h[1:] > idx_h[:-1]))))
    n_loc = int(x_dev.shape[0])
    first = max(0, m - lo)
    pick = np.unique(np.linspace(first, n_loc - 1, min(n_sample, n_loc - first)).round().astype(np.int64))
    pick = pick[~np.isin(pick + lo, idx_h)]
    ms = canon_maxcos(x_dev[torch.from_numpy(pick).to(x_dev.device)].float().cpu().numpy().astype(np.float64),
                      lab_host64)
    kth, kth_i = sc_h[-1], idx_h[-1]
    no_better = bool(np.all((ms > kth) | ((ms == kth) & (pick + lo > kth_i))))
    return {"selected_scores_equal_canonical_fp64": exact, "selection_sorted": sorted_ok,
            "no_sampled_row_beats_kth": no_better, "sampled_rows": int(pick.size), "k": int(k),
            "note": "host numpy fp64 restatement (sequential norms and dots) on the bf16 values"}


def bench_div(args, steps, warmup, world, rank, dev, dist, backend, cpu=12.0):
    """Config 5: one step = max-cosine of every pool row to the labeled set
    (bf16 MFMA, fp32 accumulate) + exact top-k of the least similar rows."""
    import torch

    from dal import _lib, parallel
    from dal.engine import _ptr, _stream
    from dal.similarity import LabeledSet, diversity_select

    cfg = CONFIGS["5"]
    n, d, k, m = cfg["n"], cfg["d"], cfg["k"], cfg["m"]
    lo, hi, _ = parallel.shard_range(n, world, rank)
    x = upload(host_pool(lo, hi, d, cfg["dist"]), dev).to(torch.bfloat16)
    lab_host = host_pool(0, m, d, cfg["dist"])
    lab = upload(lab_host, dev).to(torch.bfloat16)
    cand = torch.arange(max(lo, m), hi, device=dev, dtype=torch.int64)
    sharded = world > 1 or SHARDED
    comm = parallel.TorchComm() if sharded else None
    tdev = dev if backend == "nccl" else "cpu"

    def step():
        if sharded:
            return parallel.diversity_select_sharded(x, lo, lab, k, comm, candidates=cand, device=dev)
        s = diversity_select(x, None, k, candidates=cand, device=dev, labeled_rows=lab)
        return s.indices, s.selected_scores

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(warmup):
        step()
    elapsed, (sel_idx, sel_sc) = _timed(step, steps, barrier)
    check = div_self_check(x, upload(lab_host, dev).to(torch.bfloat16).float().cpu().numpy().astype(np.float64),
                           lo, m, sel_idx, sel_sc, k) if world == 1 else None
    if check is not None and not (check["selected_scores_equal_canonical_fp64"] and check["selection_sorted"]
                                  and check["no_sampled_row_beats_kth"]):
        raise SystemExit(f"bench self-check FAILED (config 5): {check}")
    # kernel-only timing of the max-cosine launch on this rank
    L = LabeledSet(lab, dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.empty(hi - lo, dtype=torch.float32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def launch():
        _lib.call("dal_max_cosine_unit", _ptr(x), hi - lo, d, _ptr(L.unit16), L.m_pad, _ptr(out), _ptr(st),
                  _stream(dev))

    # back-to-back launches between two events (an event pair around each
    # launch also times the host's submission of that launch), after 30
    # untimed ones: the host-side self-check leaves the GPU idle and its clock
    # takes tens of milliseconds to ramp back (first 5-launch window 1.69 ms
    # vs 1.42-1.44 ms held, scripts/maxcos_window_probe.py)
    reps = 20
    for _ in range(30):
        launch()
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    kms = e0.elapsed_time(e1) / reps
    elapsed, _ = _max_over_ranks([elapsed, kms], world, dist, tdev)
    flops = 2.0 * (hi - lo) * m * d
    achieved = flops / (kms * 1e-3) / 1e12
    res = {
        "metric": "pool rows scored/sec (diversity: max-cosine to labeled set + exact top-k)",
        "value": (n - m) * steps / elapsed, "unit": "rows/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": elapsed * 1000 / steps, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None,
        "dtype": "bf16 pool (rows rescaled by powers of two to fp16 exactly; fp16 MFMA, fp32 accumulate)",
        "data": DATA_NOTE,
        "config": {"workload": cfg["workload"], "pool_rows": n, "features": d, "labeled": m, "k": k,
                   "parallelism": f"row-shard dp{world}" if sharded else "single GPU"},
        "roofline": {"bound": "mfma", "kernel": "dal_max_cosine_unit (bf16 pool rows power-of-two scaled to fp16 in registers, folded fp16 unit labeled rows; v_mfma_f32_16x16x32_f16, max-only epilogue)",
                     "achieved": achieved, "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / BF16_MFMA_PEAK_TFLOPS,
                     "traffic": _traffic("5", "maxcos_bytes_per_launch", world), "launch_ms": kms,
                     "algorithmic_flops_per_launch": flops, "pool_bytes_per_launch": (hi - lo) * d * 2,
                     "hbm_frac_of_8TBs": (hi - lo) * d * 2 / (kms * 1e-3) / 8e12},
        "self_check": check,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and cpu and not args.no_cpu_baseline:
        xs = x[: 300_000].float().cpu().numpy()  # the bf16 values the GPU scores, as fp32
        res["cpu_baseline"] = cpu_baseline_div(xs, m, k, n, budget_s=float(cpu))
    return res


def bench_rf_train(dev, n: int = 5000, d: int = 64, trees: int = 10, reps: int = 20):
    """Per-iteration model fit (uncertainty_sampling.py:71-76): GPU
    RandomForest.trainClassifier on an AL-sized labeled set vs scikit-learn's
    fit on the host.  Synthetic labeled rows (U[0,1), label = thresholded row
    sum), seeded bagging draws."""
    import torch
    from sklearn.ensemble import RandomForestClassifier

    from dal.random_forest import bagging_inputs, train_classifier

    rng = np.random.default_rng(7)
    X = rng.random((n, d), dtype=np.float32)
    y = (X[:, : d // 8].sum(axis=1) > d // 16).astype(np.int64)
    w, s = bagging_inputs(n, d, trees, 4, seed=1)
    xd = torch.from_numpy(X).to(dev)
    for _ in range(3):
        train_classifier(xd, y, trees, weights=w, feature_subsets=s, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        train_classifier(xd, y, trees, weights=w, feature_subsets=s, device=dev)
    torch.cuda.synchronize()
    gpu_ms = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    RandomForestClassifier(n_estimators=trees, max_depth=4, max_features="sqrt", bootstrap=True,
                           random_state=0, n_jobs=-1).fit(X, y)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    return {"workload": f"RandomForest.trainClassifier on {n} x {d} labeled rows, T={trees}, depth 4, "
                        "32 bins, sqrt features (MLlib 2.1 algorithm)",
            "gpu_ms_per_fit": gpu_ms, "sklearn_host_ms_per_fit": cpu_ms, "cores": _cores(),
            "note": "wall per fit incl. the host's bagging draws and the forest's copy back; sklearn is "
                    "a different (midpoint-threshold) algorithm timed for scale"}


# ------------------------------------------------------------- output --
HEADLINE_MAX_BYTES = 4000
EXTRA_MAX_BYTES = 1024


def _r(v, nd=4):
    """A float rounded to ``nd`` significant digits (None passes)."""
    if v is None or isinstance(v, (bool, int, str)):
        return v
    return float(f"{float(v):.{nd}g}")


def _roof_short(r, keys=("bound", "achieved", "peak", "unit", "frac", "traffic", "launch_ms",
                         "fused_step_select_ms", "used_features")):
    if not r:
        return None
    return {k: _r(r.get(k), 5 if k in ("frac", "launch_ms", "fused_step_select_ms") else 4) for k in keys
            if k in r}


def _checks(sc):
    """The boolean self-checks of a result (names kept, notes dropped)."""
    if not sc:
        return None
    return {k: v for k, v in sc.items() if isinstance(v, bool) or v is None}


def headline(out: dict) -> dict:
    """The driver-parsed last stdout line: the contract's keys, numbers only
    in the sub-objects, short kernel names; everything else stays in the full
    result file."""
    h = {k: out.get(k) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data")}
    cfg = out.get("config") or {}
    h["config"] = {k: cfg[k] for k in ("workload", "pool_rows", "features", "trees", "k", "labeled",
                                       "parallelism") if k in cfg}
    for k in ("world_size", "backend", "sharded_path"):
        h[k] = out.get(k)
    h["value"], h["ms_per_step"] = _r(out.get("value"), 6), _r(out.get("ms_per_step"), 6)
    h["warm_selection_latency_ms"] = _r(out.get("warm_selection_latency_ms"))
    h["self_check"] = _checks(out.get("self_check"))
    roof = out.get("roofline") or {}
    h["roofline"] = dict(_roof_short(roof) or {}, kernel=str(roof.get("kernel", ""))[:80],
                         launch_ms_max_over_ranks=_r(roof.get("launch_ms_max_over_ranks"), 5),
                         algorithmic_flops_per_launch=_r(roof.get("algorithmic_flops_per_launch"), 6))
    h["roofline_forest"] = _roof_short(out.get("roofline_forest"))
    h["roofline_topk"] = _roof_short(out.get("roofline_topk"))
    cb = out.get("cpu_baseline")
    h["cpu_baseline"] = None if not cb else {"value": _r(cb.get("value")), "unit": cb.get("unit"),
                                             "cores": cb.get("cores"), "kind": cb.get("kind"),
                                             "sample": str(cb.get("sample", ""))[:160]}
    acc = out.get("accuracy") or {}
    if acc:
        h["accuracy"] = {k: _r(acc.get(k), 3) for k in ("density_max_rel_err", "density_err_bound_rel",
                                                         "kth_gap_rel") if k in acc}
    if out.get("ranks"):
        h["ranks"] = {k: _r(v) for k, v in out["ranks"].items()}
    if out.get("full_result"):
        h["full_result"] = out["full_result"]
    return h


def extra_line(label: str, r: dict) -> dict:
    """One extra workload as a short JSON object (printed before the headline)."""
    if "gpu_ms_per_fit" in r:  # rf_train
        return {"extra": label, "gpu_ms_per_fit": _r(r["gpu_ms_per_fit"]),
                "sklearn_host_ms_per_fit": _r(r["sklearn_host_ms_per_fit"]), "cores": r.get("cores")}
    cfg = r.get("config") or {}
    e = {"extra": label, "value": _r(r.get("value"), 5), "unit": r.get("unit"),
         "ms_per_step": _r(r.get("ms_per_step"), 5), "steps": r.get("steps"),
         "shape": f"{cfg.get('pool_rows')}x{cfg.get('features')}"
                  + (f" T={cfg['trees']}" if "trees" in cfg else "") + f" k={cfg.get('k')}"
                  + (f" m={cfg['labeled']}" if "labeled" in cfg else ""),
         "warm_ms": _r(r.get("warm_selection_latency_ms"))}
    for key, short in (("roofline", "gram"), ("roofline_forest", "forest"), ("roofline_topk", "topk")):
        ro = r.get(key)
        if ro:
            e[short] = {"frac": _r(ro.get("frac")), "ms": _r(ro.get("launch_ms")), "bound": ro.get("bound")}
            if ro.get("fused_step_select_ms"):
                e[short]["fused_ms"] = _r(ro["fused_step_select_ms"])
    if "gram" in e and str(r["roofline"].get("kernel", "")).startswith("dal_max_cosine"):
        e["maxcos"] = e.pop("gram")
    cb = r.get("cpu_baseline")
    if cb:
        e["cpu_rows_per_s"] = _r(cb.get("value"))
    sc = _checks(r.get("self_check"))
    if sc is not None:
        e["self_check_ok"] = all(v for v in sc.values() if v is not None)
    acc = r.get("accuracy") or {}
    if "density_max_rel_err" in acc:
        e["density_max_rel_err"] = _r(acc["density_max_rel_err"], 3)
    if acc.get("density_max_err_over_abs_rowsum") is not None:  # signed pools (config 3)
        e["density_err_over_abs_rowsum"] = _r(acc["density_max_err_over_abs_rowsum"], 3)
    return e


def emit(out: dict, path: str | None):
    """Write the full result to ``path`` and print the extras, then the
    headline LAST (rank 0 only)."""
    if path:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            with open(path, "w") as f:
                json.dump(out, f, indent=1)
            out = dict(out, full_result=os.path.relpath(os.path.abspath(path), REPO))
        except OSError as e:  # the headline still prints
            print(f"bench: could not write {path}: {e}", file=sys.stderr)
    for label, r in (out.get("extra") or {}).items():
        print(json.dumps(extra_line(label, r), separators=(",", ":")), flush=True)
    print(json.dumps(headline(out)), flush=True)


# ------------------------------------------------------------ launcher --
def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int, cmd: list, env: dict | None = None, poll_s: float = 0.05) -> int:
    """Run ``cmd`` as ``n`` ranks of one node (the self-launch of
    ``bench.py --gpus N`` when no outside launcher set WORLD_SIZE).

    The parent never touches the GPU: it starts ``n`` child processes (never an
    exec of itself) with RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE and a
    127.0.0.1 rendezvous, forwards rank 0's stdout line by line to its own
    stdout (so rank 0's headline stays the LAST stdout line) and every other
    rank's stdout to stderr.  When a rank exits nonzero the others are
    terminated (they would wait in a collective) and the parent returns that
    rank's exit code (a signal -s as 128 + s); 0 when all ranks exit 0."""
    import subprocess
    import threading

    base = dict(os.environ if env is None else env)
    base.setdefault("MASTER_ADDR", "127.0.0.1")
    base["MASTER_PORT"] = str(base.get("DAL_BENCH_MASTER_PORT") or _free_port())
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", ROLE_RANK=str(r))
        procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE, text=True, bufsize=1))

    def pump(p, dst):
        for line in p.stdout:
            dst.write(line)
            dst.flush()

    pumps = [threading.Thread(target=pump, args=(p, sys.stdout if r == 0 else sys.stderr), daemon=True)
             for r, p in enumerate(procs)]
    for t in pumps:
        t.start()
    rc = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench launcher: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    procs[q].terminate()
        if live:
            time.sleep(poll_s)
    for r, p in enumerate(procs):
        if p.returncode is None:  # (terminated above and still not reaped)
            p.kill()
            p.wait()
    for t in pumps:
        t.join(timeout=10)
    return rc


def main():
    # --gpus N > 1 without an outside launcher (no WORLD_SIZE in the
    # environment): start N ranks as child processes before anything here
    # touches torch or the GPU, and exit with their status
    if "WORLD_SIZE" not in os.environ:
        pre = argparse.ArgumentParser(add_help=False)
        pre.add_argument("--gpus", type=int, default=1)
        ngpus = pre.parse_known_args()[0].gpus
        if ngpus > 1:
            sys.exit(launch_ranks(ngpus, [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: config 4: 5, else 50)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default: config 4: 1, else 10)")
    ap.add_argument("--config", default="4", choices=sorted(CONFIGS))
    ap.add_argument("--extra", default=None,
                    help="comma list of extra configs reported under 'extra' (default: '2' with config 4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--warm-steps", type=int, default=None)
    ap.add_argument("--trees", type=int, default=None, help="override the config's forest size (config 4: T=100)")
    ap.add_argument("--k", type=int, default=None, help="override the config's selection size (config 4: k=1000)")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "bench_full.json"),
                    help="file for the full result (every note and sub-field); '' to skip")
    args = ap.parse_args()
    main_cfg = resolve(f"{args.config}" + (f":T{args.trees}" if args.trees is not None else "")
                       + (f":k{args.k}" if args.k is not None else ""))[1]
    big = args.config in ("4",)
    steps = args.steps if args.steps is not None else (5 if big else 50)
    warmup = args.warmup if args.warmup is not None else (1 if big else 10)
    warm_steps = args.warm_steps if args.warm_steps is not None else (5 if big else 20)
    extra = args.extra if args.extra is not None else (DEFAULT_EXTRA if args.config == "4" and
                                                        args.trees is None and args.k is None else "")
    extra = [c for c in extra.split(",") if c and c != "none"]

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:  # (an outside launcher set a different WORLD_SIZE)
        raise SystemExit(f"--gpus {args.gpus} but the launcher's WORLD_SIZE={world}")
    # DAL_BENCH_BACKEND=gloo rehearses the multi-process path with several
    # ranks on one GPU (all-gathers staged through the host); default: RCCL.
    backend = os.environ.get("DAL_BENCH_BACKEND", "nccl")
    n_dev = torch.cuda.device_count()
    dev = torch.device("cuda", local_rank % max(n_dev, 1))
    torch.cuda.set_device(dev)
    if world > 1 or SHARDED:
        if world == 1:  # DAL_BENCH_SHARDED=1: a one-rank group of its own
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)

    if main_cfg.get("mode") == "div":
        out = bench_div(args, steps, warmup, world, rank, dev, dist, backend)
    else:
        out = bench_dw(args, args.config, steps, warmup, warm_steps, world, rank, dev, dist, backend, cfg=main_cfg)
    if extra:
        out["extra"] = {}
        for spec in extra:
            c, cfg, label = resolve(spec)
            t0 = time.perf_counter()
            variant = ":" in spec  # config-4 T=100 / k=1000: the same 2M x 256 pool, fewer steps
            # 60 untimed steps (0.06-0.25 s of GPU work): after the previous
            # config's host-side checks the clock needs tens of milliseconds
            # to ramp back, longer than 5 steps of a 1-4 ms config
            if cfg.get("mode") == "div":
                r = bench_div(args, 20, 60, world, rank, dev, dist, backend, cpu=8.0)
            elif variant:
                r = bench_dw(args, c, 3, 1, 5, world, rank, dev, dist, backend, cpu=False, cfg=cfg)
            else:
                r = bench_dw(args, c, 20, 60, 20, world, rank, dev, dist, backend, cpu=8.0, cfg=cfg)
            out["extra"][label] = {kk: r[kk] for kk in (
                "metric", "value", "unit", "steps", "warmup", "ms_per_step", "dtype", "config",
                "warm_selection_latency_ms", "self_check", "accuracy", "roofline", "roofline_forest",
                "roofline_topk", "cpu_baseline") if kk in r}
            out["extra"][label]["wall_s"] = time.perf_counter() - t0
            if variant:
                out["extra"][label]["cpu_baseline_note"] = ("the host cost of this variant is the headline "
                                                            "line's O(N^2) Gram row-sum (cpu_baseline above)")
    if world == 1 and CONFIGS[args.config].get("mode") != "div":
        out.setdefault("extra", {})["rf_train"] = bench_rf_train(dev)
    out["world_size"] = dist.get_world_size() if world > 1 or SHARDED else 1
    out["backend"] = dist.get_backend() if world > 1 or SHARDED else None
    out["sharded_path"] = bool(world > 1 or SHARDED)
    if rank == 0:
        emit(out, args.out)
    if world > 1 or SHARDED:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
