"""Row-sharded multi-GPU query selection (one process per GPU, RCCL over xGMI).

Reference parallelism: Spark data parallelism over RDD row partitions, with
the cross-partition steps done as shuffles:
BlockMatrix.multiply's block cogroup (density_weighting.py:73), groupByKey
(:144, :159) and sortBy + take to the driver (:168, :172).

Here the pool is row-sharded in contiguous shards of ``shard`` rows (a
multiple of DAL_ROW_GRANULE, identical on every rank; the last rank holds the
remainder).  Two exchanges, both all-gathers over ``torch.distributed``
(backend "nccl" = RCCL on ROCm):

  1. the shards' Gram operands (fp16 split [shard, 2*d_pad] by default, or
     fp32 unit rows) and the canonical fp64 column-sum partials -> every rank
     holds U (the density needs every column; the symmetric kernel's
     closed-form remainder needs every super block's row sums) -- replaces
     the BlockMatrix shuffle.  The operand all-gather runs asynchronously on RCCL's stream
     while each rank multiplies its rows by its OWN shard's columns (CUs
     reserved for RCCL), then by the rest (ShardedSelector.exchange_density);
  2. each rank's exact local top-k (key, index, score) -> an identical
     deterministic merge on every rank -- replaces sortBy + take.

Determinism: global row r sits at column r of the gathered U on every P, the
density is accumulated in exact int64 fixed point, and the canonical column
sum is reduced over the same 256-row chunks in the same order, so every
density bit, every score and the selected set are identical for P = 1..8.

The phases are methods so that tests can drive P shards in one process
(GPU, ``emulate``) or replace the local HIP steps with the oracle (CPU, gloo).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import DAL_ASCENDING, DAL_CANON_CHUNK, DAL_DESCENDING, DAL_KEY_NONE, DAL_ROW_GRANULE

# CUs left to RCCL while the own-shard Gram launch runs beside the all-gather
# (a persistent Gram grid would otherwise hold every CU's registers and LDS).
RCCL_RESERVED_CUS = 8


def shard_rows(n_total: int, world: int) -> int:
    """Rows per shard: ceil(N / P) rounded up to the row granule (512)."""
    per = -(-n_total // world)
    return -(-per // DAL_ROW_GRANULE) * DAL_ROW_GRANULE


def shard_range(n_total: int, world: int, rank: int):
    s = shard_rows(n_total, world)
    lo = min(rank * s, n_total)
    hi = min(lo + s, n_total)
    return lo, hi, s


@dataclass
class LocalTopk:
    """A rank's exact local top-k, padded to k with DAL_KEY_NONE."""

    keys: object  # int64 [k] (uint64 bit patterns)
    idx: object  # int64 [k] global row indices
    scores: object  # fp64 [k]


def merge_topk(keys_all, idx_all, scores_all, k: int, sort_fn, all_valid: bool = False):
    """Deterministic merge of P gathered local top-k lists (rank-major).

    Each list is sorted by (key, index) and shards are in global index order,
    so sorting by (key, position) orders ties by global index; ``sort_fn``
    returns the positions of the k best.  ``all_valid``: at least k candidates
    exist globally, so no padding key can reach the k best and the filter
    (a host sync) is skipped."""
    torch = __import__("torch")
    n = int(keys_all.shape[0])
    pos = torch.arange(n, dtype=torch.int64, device=keys_all.device)
    best = sort_fn(keys_all, pos, k)
    if not all_valid:
        valid = keys_all[best] != _as_i64(DAL_KEY_NONE)
        best = best[valid]
    return idx_all[best], scores_all[best]


def _as_i64(u: int) -> int:
    return u - (1 << 64) if u >= (1 << 63) else u


class ShardedSelector:
    """One rank's shard of the pool and its share of a selection step."""

    def __init__(self, x_local, n_total: int, rank: int, world: int, excluded=None, device=None,
                 gram: str = None):
        from .engine import PoolState

        self.n_total, self.rank, self.world = int(n_total), int(rank), int(world)
        self.lo, self.hi, self.shard = shard_range(self.n_total, self.world, self.rank)
        if int(x_local.shape[0]) != self.hi - self.lo:
            raise ValueError(f"rank {rank}: expected {self.hi - self.lo} rows, got {x_local.shape[0]}")
        self.state = PoolState(x_local, excluded=excluded, device=device, row_base=self.lo,
                               n_total=self.n_total, n_pad=self.shard, gram=gram)
        self._density = None
        self._parts_full = None  # all ranks' canonical column-sum partials (cached with the density)
        self._colsum = None      # the global canonical column sum reduced from them (cached)
        self._plans = {}         # warm-step plans by (T, depth, k, beta, cap, level-1 passes)
        self.cap_scale = 1      # re-rank candidate capacity multiplier (grown on overflow)
        # bench: list -> (name, start, end) HIP events around the density
        # exchange's collective ("all_gather": operand + partials, recorded on
        # the stream that waits for them)
        self.exchange_events = None

    def index_tensor(self, unlabeled_idx):
        from .engine import _as_index

        return _as_index(unlabeled_idx, self.state.device)

    def status_word(self):
        """This rank's device status word (DAL_FLAG_* bits), int32 [1]."""
        return self.state.status

    def prepare_retry(self, sample_miss: bool = False):
        """After a re-rank capacity overflow (or a fast level-1
        overflow) anywhere: grow the capacity (or fall back to the exact radix
        level 1) and go again.  The density, operand and column-sum caches stay valid,
        so the retry does not redo the Gram."""
        self.state.status.zero_()
        if sample_miss:
            self.state.level1_fast = False
        else:
            self.cap_scale *= 4

    def clear_caches(self):
        """Drop the shard's normalised rows, density and column sums (cold step)."""
        self.state.clear_caches()
        self._density = None
        self._parts_full = None
        self._colsum = None
        self._plans = {}

    def global_colsum(self, partials_full):
        """The canonical column sum s = sum_{j not in E} u_j over EVERY rank's
        rows, reduced once from the gathered partials and cached (a warm-step
        plan captures its address)."""
        if self._colsum is None or partials_full is not self._parts_full:
            cs = self.state.colsum(partials_full)
            if partials_full is not self._parts_full:
                return cs
            self._colsum = cs
        return self._colsum

    def warm_plan(self, forest, k: int, beta: float):
        """This rank's warm local step (density cached) as a dal_dw_plan whose
        outputs land in one packed row [keys k | indices k | score bits k |
        status]: launched without a host wait, all-gathered and merged
        stream-ordered (engine.WarmStepGraph with ``packed``)."""
        from .engine import WarmStepGraph, candidate_cap, level1_passes

        torch = __import__("torch")
        st = self.state
        base = candidate_cap(st.n, k) if st.cap_base is None else max(int(k), int(st.cap_base))
        cap = int(min(st.n, base * self.cap_scale))
        passes = level1_passes(st, st.n, k, cap)
        key = (forest.n_trees, forest.depth, int(k), float(beta), cap, passes)
        g = self._plans.get(key)
        if g is None:
            packed = torch.empty(3 * int(k) + 1, dtype=torch.int64, device=st.device)
            g = self._plans[key] = WarmStepGraph(st, forest, int(k), beta, cap, passes,
                                                 colsum=self.global_colsum(self._parts_full), packed=packed)
        return g

    # ---- phase A: local normalisation + canonical partials ------------
    def prep(self):
        """(Gram operand of the shard -- fp32 unit rows [shard, d_pad] or their
        fp16 split [shard, 2*d_pad] --, partials [shard/256, d] fp64)."""
        torch = __import__("torch")
        st = self.state
        u = st.gram_operand()
        parts = torch.zeros((self.shard // DAL_CANON_CHUNK, st.d), dtype=torch.float64,
                            device=st.device)
        if st.n:
            p = st.colsum_partials()
            parts[: p.shape[0]] = p
        return u, parts

    # ---- exchange 1 overlapped with the own-shard columns ---------------
    def exchange_density(self, comm, u_local, parts=None, reserve_cus: int = RCCL_RESERVED_CUS):
        """All-gather the shards' Gram operands (and the canonical partials)
        while this rank's rows run against its OWN columns (the operand it
        already holds), then against the other shards' columns; returns
        (gathered operand, gathered partials).  Every column range is a whole
        number of shards (multiples of 512), so the exact fixed-point sum is the
        same bits as one call over all columns.

        With RCCL (``comm.overlaps``) the own-shard Gram is queued FIRST, on
        all but ``reserve_cus`` CUs, and the collectives are enqueued behind it
        from a side stream that only waits for the operand -- the host's
        collective-issue time runs under the Gram instead of in front of it.
        gram "sym": the accumulator is indexed by global row; this rank's
        pairs yield row sums of its own rows only (the column sums of the pairs
        that take its rows come from the closed-form residual), so no density
        collective follows the all-gather."""
        torch = __import__("torch")
        st = self.state
        acc = self._new_acc()
        if getattr(comm, "overlaps", False) and st.n:
            main = torch.cuda.current_stream(st.device)
            ready = main.record_event()
            grid = max(1, 2 * (_device_cus(st.device) - reserve_cus))
            st.gram_accumulate(acc, u_local, self.shard, grid_blocks=grid, col_row0=self.lo)
            side = _side_stream(st.device)
            side.wait_event(ready)
            with torch.cuda.stream(side):
                ev = self._event_start("all_gather")
                parts_full, pwork = comm.all_gather_start(parts) if parts is not None else (None, None)
                u_full, work = comm.all_gather_start(u_local)
                if ev is not None:  # the side stream waits for the collectives, then records
                    comm.wait(work)
                    comm.wait(pwork)
                    self._event_end(ev)
            for t in (u_full, parts_full):
                if t is not None:
                    t.record_stream(main)
            main.wait_stream(side)
            comm.wait(work)   # the current (main) stream waits for the collectives
            comm.wait(pwork)
        else:
            ev = self._event_start("all_gather")
            parts_full, pwork = comm.all_gather_start(parts) if parts is not None else (None, None)
            u_full, work = comm.all_gather_start(u_local)
            if ev is not None:
                if work is None and pwork is None:  # staged (gloo): already complete
                    self._event_end(ev)
                else:  # the end on a side stream that waits for the collectives only (not the Gram below)
                    side = _side_stream(st.device)
                    side.wait_stream(torch.cuda.current_stream(st.device))
                    with torch.cuda.stream(side):
                        comm.wait(work)
                        comm.wait(pwork)
                        self._event_end(ev)
                ev = None
            if st.n:
                st.gram_accumulate(acc, u_local, self.shard, col_row0=self.lo)
            comm.wait(work)
            comm.wait(pwork)
        if st.n and self.world > 1:
            if st.gram == "sym":  # one launch over every other column
                st.gram_accumulate(acc, u_full, self.world * self.shard, col_row0=0,
                                   skip=(self.lo, self.lo + self.shard))
            else:
                for c0, c1 in other_column_ranges(self.rank, self.world, self.shard):
                    st.gram_accumulate(acc, u_full[c0:c1], c1 - c0, col_row0=c0)
        if st.gram == "sym":
            if st.n:  # the closed-form remainder and column sums of this rank's rows
                st.gram_residual(acc, u_full)
            acc = self._own_rows(acc)
        self.set_density(acc)
        return u_full, parts_full

    def _own_rows(self, acc):
        """gram "sym": the kernel adds the row sums of the pairs this rank's
        super blocks take and the residual adds every other part of its rows
        (the column sums of the pairs that take them, in closed form), all at
        GLOBAL row indices of a [world * shard] accumulator -- nothing lands on
        another rank's rows, so the density is this rank's slice (no
        collective)."""
        return acc[self.rank * self.shard:(self.rank + 1) * self.shard]

    def _event_start(self, name):
        if self.exchange_events is None:
            return None
        torch = __import__("torch")
        ev = (name, torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[1].record()
        return ev

    def _event_end(self, ev):
        if ev is not None:
            ev[2].record()
            self.exchange_events.append(ev)

    def _new_acc(self):
        torch = __import__("torch")
        n = self.world * self.shard if self.state.gram == "sym" else self.state.n_pad
        return torch.zeros(n, dtype=torch.int64, device=self.state.device)

    def density_contribution(self, u_full):
        """This rank's fixed-point density against every column of the
        gathered operand: its own rows' sums ([shard])."""
        acc = self._new_acc()
        if self.state.n:
            self.state.gram_accumulate(acc, u_full, int(u_full.shape[0]), col_row0=0)
            if self.state.gram == "sym":
                self.state.gram_residual(acc, u_full)
        return self._own_rows(acc) if self.state.gram == "sym" else acc

    def set_density(self, acc_local):
        self._density = acc_local
        self.state.set_density_fixed(acc_local)

    # ---- phase B: density against all columns + local exact top-k ------
    def local_density(self, u_full):
        if self._density is None:
            self.set_density(self.density_contribution(u_full))
        return self._density

    def local_select(self, u_full, partials_full, unlabeled_idx, forest, k: int, mode: str = "dw",
                     strategy: str = "least_confidence", beta: float = 1.0,
                     density_mode: str = "gram", warm: bool = None) -> LocalTopk:
        """This rank's exact local top-k.  ``warm``: the density was cached
        before this step (the score kernel then reads the shard's blocked
        copy, as the single-GPU warm step does; a cold step keeps the
        row-major kernel and builds no copy).  None: cached now."""
        from .engine import (density_error, device_lut, dw_select_local, dw_step_local, forest_score,
                             topk_keys, uncertainty_blocked)
        from .luts import ASCENDING

        torch = __import__("torch")
        st = self.state

        def empty():
            return LocalTopk(torch.full((k,), _as_i64(DAL_KEY_NONE), dtype=torch.int64, device=st.device),
                             torch.full((k,), -1, dtype=torch.int64, device=st.device),
                             torch.full((k,), float("nan"), dtype=torch.float64, device=st.device))

        if st.n == 0:
            return empty()
        flags, unl, _ = st.row_flags(unlabeled_idx)
        # no host count of this shard's candidates (a sync): rows that are not
        # candidates carry the padding key, so with fewer than k candidates
        # they fill the local list last and never survive a merge that has k
        kk = min(k, st.n)
        if mode == "dw" and density_mode == "separable":
            colsum = self.global_colsum(partials_full)
            lut_dev = device_lut("entropy", forest.n_trees, st.device)
            votes, sc, kys, _ = forest_score(st, forest, lut_dev, flags, DAL_DESCENDING,
                                             density=st.density_exact(colsum), beta=beta)
            i, kk_keys = topk_keys(kys, kk, st.row_base)
            s = sc[i - st.row_base]
        elif mode == "dw":
            # warm (density cached): the score kernel reads the shard's blocked copy, as on one GPU
            warm_now = self._density is not None if warm is None else warm
            xb = st.blocked_pool(forest) if warm_now else None
            dens = self.local_density(u_full)
            colsum = self.global_colsum(partials_full)
            lut_dev = device_lut("entropy", forest.n_trees, st.device)
            if st.events_off():  # one fused call (dal_dw_step), as the single-GPU step
                _, _, i, s, kk_keys = dw_step_local(st, forest, flags, dens, lut_dev, kk, beta, colsum,
                                                    cap_scale=self.cap_scale, sync=False, xb=xb)
            else:  # bench per-kernel timing: K2 and K3 as separate calls
                votes, sc, klo, khi = forest_score(st, forest, lut_dev, flags, DAL_DESCENDING, density=dens,
                                                   density_err=density_error(st), beta=beta, want_hi=True,
                                                   xb=xb)
                i, s, kk_keys = dw_select_local(st, flags, votes, klo, khi, lut_dev, kk, beta, colsum,
                                                cap_scale=self.cap_scale, sync=False)
        else:
            order = DAL_ASCENDING if ASCENDING[strategy] else DAL_DESCENDING
            lut_dev = device_lut(strategy, forest.n_trees, st.device)
            votes, sc, kys, _ = forest_score(st, forest, lut_dev, flags, order, xb=uncertainty_blocked(st, forest))
            i, kk_keys = topk_keys(kys, kk, st.row_base)
            s = sc[i - st.row_base]
        if kk == k:  # every slot written by the selection
            return LocalTopk(kk_keys, i, s)
        out = empty()
        out.keys[:kk], out.idx[:kk], out.scores[:kk] = kk_keys, i, s
        return out


def other_column_ranges(rank: int, world: int, shard: int):
    """Column ranges [c0, c1) of the gathered operand outside this rank's own
    shard (at most two contiguous ranges: before and after it)."""
    out = []
    if rank > 0:
        out.append((0, rank * shard))
    if rank < world - 1:
        out.append(((rank + 1) * shard, world * shard))
    return out


def _device_cus(device) -> int:
    torch = __import__("torch")
    return int(torch.cuda.get_device_properties(device).multi_processor_count)


def hip_sort_positions(keys, pos, k):
    from .engine import sort_pairs

    _, out_pos, _ = sort_pairs(keys, pos, k)
    return out_pos


def _needs_bytes(dtype) -> bool:
    """Neither RCCL/NCCL nor gloo has torch's 16-bit integer or unsigned
    16/32/64-bit types (the split Gram operand is int16 bit patterns): such
    tensors are gathered as their bytes (a gather only moves bits)."""
    torch = __import__("torch")
    names = ("int16", "uint16", "uint32", "uint64")
    return any(getattr(torch, n, None) == dtype for n in names)


_SIDE_STREAMS = {}


def _side_stream(device):
    """A second stream per device from which collectives are enqueued behind
    an already queued Gram launch."""
    torch = __import__("torch")
    key = str(device)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return _SIDE_STREAMS[key]


class TorchComm:
    """all-gather over torch.distributed (RCCL on ROCm GPUs, gloo on CPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        # RCCL collectives are asynchronous on their own stream: they can run
        # beside a Gram launch (gloo stages through the host synchronously)
        self.overlaps = self.backend == "nccl"
        self._rows = {}  # (width, device) -> the merge's gathered-rows buffer

    def all_gather_rows(self, row):
        """All-gather one int64 row per rank into a buffer kept for the next
        step ([P, w]; its previous contents were consumed by the previous
        merge, which the step's status read waited for).  The warm multi-GPU
        step's collective, with the fewest host calls (RCCL: enqueued on the
        communicator's stream, ordered before the current stream's next work)."""
        torch = __import__("torch")
        if not row.is_cuda or self.backend == "gloo":
            return self.all_gather(row.reshape(1, -1))
        w = int(row.shape[0])
        key = (w, row.device)
        out = self._rows.get(key)
        if out is None:
            out = self._rows[key] = torch.empty((self.world, w), dtype=row.dtype, device=row.device)
        self.dist.all_gather_into_tensor(out, row, group=self.group)
        return out

    def all_gather(self, t):
        out, work = self.all_gather_start(t)
        self.wait(work)
        return out

    def all_gather_start(self, t):
        """Start an all-gather; returns (output, work handle or None).  With
        RCCL it runs asynchronously on the communicator's stream."""
        torch = __import__("torch")
        if t.dim() and _needs_bytes(t.dtype):
            out, work = self.all_gather_start(t.contiguous().view(torch.uint8))
            return out.view(t.dtype), work
        if t.is_cuda and self.backend == "gloo":
            # rehearsal path (several ranks sharing one GPU): stage through the host
            return self.all_gather(t.cpu()).to(t.device), None
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if t.is_cuda:
            work = self.dist.all_gather_into_tensor(out, t.contiguous(), group=self.group, async_op=True)
            return out, work
        self.dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out, None

    def wait(self, work):
        """Order the current stream after the collective (no host block)."""
        if work is not None:
            work.wait()


def select(sel: ShardedSelector, comm, unlabeled_idx, forest, k: int, mode: str = "dw",
           strategy: str = "least_confidence", beta: float = 1.0, sort_fn=hip_sort_positions,
           density_mode: str = "gram"):
    """One selection step across all ranks; returns (indices [k], scores [k]),
    identical on every rank."""
    unl = sel.index_tensor(unlabeled_idx)
    u_full = parts_full = None
    warm = sel._density is not None  # (a cold step's score kernel keeps the row-major pool)
    if mode == "dw":  # uncertainty sampling never normalises (no density, no zero-norm check)
        need_u = density_mode == "gram" and sel._density is None
        if need_u or sel._parts_full is None:
            u_local, parts = sel.prep()
            if need_u:  # the (small) canonical partials travel with the operand, beside the Gram
                u_full, parts_full = sel.exchange_density(comm, u_local, parts)
            else:
                parts_full = comm.all_gather(parts)
            sel._parts_full = parts_full
            sel._colsum = None  # derived from the partials, as the plans' captured column sum
            sel._plans = {}
        parts_full = sel._parts_full
    n_unl_global = int(unl.shape[0])  # single source of truth for the candidate count
    stt = getattr(sel, "state", None)  # (the CPU tests' oracle shards have none)
    if (stt is not None and mode == "dw" and density_mode == "gram" and u_full is None
            and sel._density is not None and sort_fn is hip_sort_positions and sel.world * k <= _lib.DAL_SORT_CAP and stt.use_graphs
            and stt.events_off() and stt.n >= k and unl.is_cuda):
        # warm step (density cached): the local step is one plan replay whose
        # outputs ARE the packed all-gather row; no host wait before the merge
        plan = sel.warm_plan(forest, k, beta)
        plan.launch(forest, unl)
        out, st = merge_row(comm, plan.packed, k, all_valid=n_unl_global >= k)
        return _finish(sel, comm, unlabeled_idx, forest, k, mode, strategy, beta, sort_fn, density_mode, out, st)
    top = sel.local_select(u_full, parts_full, unl, forest, k, mode, strategy, beta, density_mode, warm=warm)
    # every rank's status word (zero-norm rows, re-rank capacity overflow)
    # rides in the top-k all-gather and is read once, after the merge is
    # queued: the step's one host sync, and every rank sees the same bits
    if sort_fn is hip_sort_positions and sel.world * k <= _lib.DAL_SORT_CAP and top.keys.is_cuda:
        out, st = merge_packed(comm, top, sel.status_word(), k, all_valid=n_unl_global >= k)
    else:
        keys_all, idx_all, sc_all, st_all = gather_topk(comm, top, sel.status_word())
        out = merge_topk(keys_all, idx_all, sc_all, k, sort_fn, all_valid=n_unl_global >= k)
        st = 0
        for v in st_all.tolist():
            st |= int(v)
    return _finish(sel, comm, unlabeled_idx, forest, k, mode, strategy, beta, sort_fn, density_mode, out, st)


def _finish(sel, comm, unlabeled_idx, forest, k, mode, strategy, beta, sort_fn, density_mode, out, st):
    """Act on the OR of every rank's status word (identical on all ranks)."""
    if mode != "dw":
        st &= ~_lib.DAL_FLAG_ZERO_NORM  # a zero row only matters to the cosine density
    if st & _lib.DAL_FLAG_ZERO_NORM:
        raise ValueError("pool contains a zero-norm row: cosine similarity is undefined "
                         "(the reference would propagate NaN into every density)")
    if st & (_lib.DAL_FLAG_CAND_OVERFLOW | _lib.DAL_FLAG_SAMPLE_MISS):  # rare: redo on every rank
        sel.prepare_retry(sample_miss=bool(st & _lib.DAL_FLAG_SAMPLE_MISS))
        return select(sel, comm, unlabeled_idx, forest, k, mode, strategy, beta, sort_fn, density_mode)
    return out


def gather_topk(comm, top: LocalTopk, status=None):
    """ONE all-gather of every rank's (key, index, score) triples, packed as
    int64 [3k] (scores by bit pattern), plus the rank's status word when
    given: a collective's latency, not its bytes, dominates at k = 100-1000.
    Returns (keys, idx, scores) rank-major [P*k] (+ statuses [P])."""
    torch = __import__("torch")
    k = int(top.keys.shape[0])
    parts = [top.keys, top.idx, top.scores.view(torch.int64)]
    if status is not None:
        parts.append(status.reshape(1).to(torch.int64))
    packed = torch.cat(parts)
    w = int(packed.shape[0])
    g = comm.all_gather(packed.reshape(1, w)).reshape(-1, w)              # [P, 3k (+1)]
    out = (g[:, :k].reshape(-1), g[:, k:2 * k].reshape(-1),
           g[:, 2 * k:3 * k].reshape(-1).contiguous().view(torch.float64))
    if status is not None:
        out = out + (g[:, 3 * k],)
    return out


def merge_packed(comm, top: LocalTopk, status, k: int, all_valid: bool = False):
    """gather_topk + merge_topk in one all-gather and one C call
    (dal_topk_merge reads the gathered [P, 3k+1] rows in place: unpack, sort
    by (key, rank-major position), gather; the status words OR-ed on the
    device).  Returns ((indices, scores), status) -- the status read is the
    step's one host sync."""
    torch = __import__("torch")
    packed = torch.cat([top.keys, top.idx, top.scores.view(torch.int64), status.reshape(1).to(torch.int64)])
    return merge_row(comm, packed, k, all_valid)


def merge_row(comm, packed, k: int, all_valid: bool = False):
    """All-gather this rank's packed row int64 [3k+1] (keys | indices | score
    bits | status) and merge the rows with dal_topk_merge; returns ((indices,
    scores), OR of the status words)."""
    torch = __import__("torch")
    from .engine import _ptr, _stream
    from ._lib import call

    dev = packed.device
    w = int(packed.shape[0])
    g = comm.all_gather_rows(packed) if hasattr(comm, "all_gather_rows") else comm.all_gather(packed.reshape(1, w))
    n_ranks = int(g.shape[0])
    lib = _lib.load()
    wsb = int(lib.dal_topk_merge_workspace_bytes(n_ranks, k))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev) if wsb else None  # (the one-launch merge needs none)
    # the outputs in one allocation: indices | score bits | (keys) | status
    nk = 2 if all_valid else 3
    buf = torch.empty(nk * k + 1, dtype=torch.int64, device=dev)
    b0 = buf.data_ptr()
    call("dal_topk_merge", _ptr(g), n_ranks, w, k, 0 if ws is None else _ptr(ws), wsb, b0, b0 + 8 * k,
         0 if all_valid else b0 + 16 * k, b0 + 8 * nk * k, _stream(dev))
    st = int(buf[nk * k].item()) & 0xFFFFFFFF  # the int32 status in the low half (little endian)
    st = st - (1 << 32) if st >= (1 << 31) else st
    out_idx, out_sc = buf[:k], buf[k:2 * k].view(torch.float64)
    out_keys = None if all_valid else buf[2 * k:3 * k]
    if out_keys is not None:
        valid = out_keys != _as_i64(DAL_KEY_NONE)
        out_idx, out_sc = out_idx[valid], out_sc[valid]
    return (out_idx, out_sc), st


def emulate(selectors, unlabeled_idx, forest, k: int, mode: str = "dw",
            strategy: str = "least_confidence", beta: float = 1.0, sort_fn=hip_sort_positions,
            density_mode: str = "gram"):
    """Run P shards in one process (tests): the all-gathers become concatenations."""
    torch = __import__("torch")
    u_full = parts_full = None
    if mode == "dw":  # uncertainty sampling never normalises
        preps = [s.prep() for s in selectors]
        u_full = torch.cat([p[0] for p in preps])
        parts_full = torch.cat([p[1] for p in preps])
    if mode == "dw" and density_mode == "gram" and selectors and selectors[0]._density is None:
        for s in selectors:
            s.set_density(s.density_contribution(u_full))
    tops = [s.local_select(u_full, parts_full, unlabeled_idx, forest, k, mode, strategy, beta,
                           density_mode)
            for s in selectors]
    keys_all = torch.cat([t.keys for t in tops])
    idx_all = torch.cat([t.idx for t in tops])
    sc_all = torch.cat([t.scores for t in tops])
    n_unl = int(np.asarray(unlabeled_idx).reshape(-1).shape[0]) if not hasattr(unlabeled_idx, "shape") \
        else int(unlabeled_idx.shape[0])
    out = merge_topk(keys_all, idx_all, sc_all, k, sort_fn, all_valid=n_unl >= k)
    st = 0
    for s in selectors:
        st |= int(s.state.status.item())
    if st & (_lib.DAL_FLAG_SAMPLE_MISS | _lib.DAL_FLAG_CAND_OVERFLOW):  # as select(): redo on every shard
        for s in selectors:
            s.prepare_retry(sample_miss=bool(st & _lib.DAL_FLAG_SAMPLE_MISS))
        return emulate(selectors, unlabeled_idx, forest, k, mode, strategy, beta, sort_fn, density_mode)
    for s in selectors:
        s.state.check_status()
    return out


def diversity_select_sharded(x_local, row_base: int, labeled_rows, k: int, comm, candidates=None,
                             device=None, sort_fn=hip_sort_positions):
    """Batch-mode diversity selection (BASELINE config 5) over a row-sharded
    bf16 pool: every rank scores its rows against the replicated labeled set
    (no exchange), keeps its exact local top-k, and the all-gathered lists are
    merged identically on every rank."""
    from .similarity import diversity_select

    torch = __import__("torch")
    n = int(x_local.shape[0])
    dev = x_local.device if device is None else device
    keys = torch.full((k,), _as_i64(DAL_KEY_NONE), dtype=torch.int64, device=dev)
    idx = torch.full((k,), -1, dtype=torch.int64, device=dev)
    sc = torch.full((k,), float("nan"), dtype=torch.float64, device=dev)
    if n:
        sel = diversity_select(x_local, None, k, candidates=candidates, device=dev, row_base=row_base,
                               labeled_rows=labeled_rows)
        kk = int(sel.indices.shape[0])
        idx[:kk] = sel.indices
        sc[:kk] = sel.selected_scores
        keys[:kk] = _score_keys_asc(sel.selected_scores)
    return merge_topk(*gather_topk(comm, LocalTopk(keys, idx, sc)), k, sort_fn)


def _score_keys_asc(s):
    """Ascending score keys of finite fp64 scores, computed on the device with
    the C ABI's encoding (-0 -> +0; negative -> ~bits; else bits | sign bit),
    stored as int64 bit patterns of the uint64 keys."""
    torch = __import__("torch")
    s = torch.where(s == 0, torch.zeros_like(s), s)
    b = s.view(torch.int64)
    return torch.where(b < 0, ~b, b | (-(1 << 63)))
