"""Device pipeline of one query-selection step (single GPU / one shard).

Every arithmetic step is a libdal HIP kernel (include/dal.h); torch is used
only for device memory, the current HIP stream and trivial index plumbing.
There is no CPU fallback: without libdal.so or a GPU these functions raise.

Reference loop body being replaced (one ``while True`` iteration):
  uncertainty_sampling.py:85-112   per-tree predict, vote sum, LC score, sortBy, take(k)
  density_weighting.py:58-100      proximity matrix (built once per pool)
  density_weighting.py:133-176     entropy x density, descending sortBy, take(k)
"""
from __future__ import annotations


import weakref

import numpy as np

from . import _lib
from ._lib import (DAL_ASCENDING, DAL_CANON_CHUNK, DAL_DENSITY_EXACT, DAL_DENSITY_FIXED,
                   DAL_DENSITY_NONE, DAL_DESCENDING, DAL_FIXED_SCALE, DAL_FLAG_CAND_OVERFLOW,
                   DAL_FLAG_SAMPLE_MISS, DAL_FLAG_ZERO_NORM, DAL_ROW_CANDIDATE, DAL_ROW_EXCLUDED,
                   DAL_SORT_CAP_PAYLOAD, DAL_STEP_RESET_STATUS,
                   DAL_STEP_WS_CLEAN, call)
from .forest import Forest
from .luts import ASCENDING, lut as make_lut


def _torch():
    import torch

    return torch


def _stream(device=None) -> int:
    torch = _torch()
    return torch.cuda.current_stream(device).cuda_stream


def _raw_stream(device) -> int:
    """The current HIP stream of ``device`` (an indexed torch.device) as an
    integer, without building a Stream object (warm-step host path)."""
    return _torch()._C._cuda_getCurrentRawStream(device.index)


def _ptr(t) -> int:
    return t.data_ptr()


def _require_cuda(device):
    torch = _torch()
    if not torch.cuda.is_available():
        raise _lib.DalError("dal requires a ROCm GPU (torch.cuda.is_available() is False)")
    dev = torch.device(device if device is not None else "cuda")
    if dev.type == "cuda" and dev.index is None:  # pin the index (raw stream / index checks)
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


class Selection:
    """Result of one selection step (all tensors on the pool's device).

    scores          fp64 [U]: score of every unlabeled row, in ``unlabeled`` order
    indices         int64 [k]: selected global row indices, best first
    selected_scores fp64 [k]: their scores (canonical fp64 for density weighting)
    votes           int32 [U]: forest votes for class 1 of every unlabeled row

    ``scores`` / ``votes`` may be given as (per-row tensor, positions): they are
    gathered into unlabeled order on first access (the per-row arrays are
    complete in HBM when the step returns; the gather is only a re-layout, so
    a caller that reads just the selection pays no extra launches).
    """

    def __init__(self, scores, indices, selected_scores, votes=None):
        self._scores = scores
        self.indices = indices
        self.selected_scores = selected_scores
        self._votes = votes

    @staticmethod
    def _gathered(v):
        if isinstance(v, tuple):
            full, pos = v
            return full if pos is None else full[pos]
        return v

    @property
    def scores(self):
        self._scores = self._gathered(self._scores)
        return self._scores

    @property
    def votes(self):
        self._votes = self._gathered(self._votes)
        return self._votes

    def _detach(self):
        """Materialise the per-row arrays now (their source buffers are about
        to be reused: a warm-step graph replay)."""
        self._scores = self._gathered(self._scores)
        self._votes = self._gathered(self._votes)

    def __iter__(self):
        """Unpacks as the reference-shaped triple (scores, indices, selected_scores)."""
        return iter((self.scores, self.indices, self.selected_scores))

    def __repr__(self):
        return f"Selection(indices={self.indices!r}, selected_scores={self.selected_scores!r})"

    def as_pairs(self):
        """``add_to_labeled_set`` of the reference: a list of (index, score)."""
        return list(zip(self.indices.cpu().tolist(), self.selected_scores.cpu().tolist()))


class PoolState:
    """A device-resident pool and its per-pool caches.

    The reference builds the proximity matrix once per pool and drops the
    initial labeled window L0 from it once (density_weighting.py:58-100), so the
    density is constant across AL iterations; it is computed lazily here and
    cached (the "warm" path), keyed by the excluded set.

    For a row shard (multi-GPU) ``row_base`` is the global index of row 0 and
    ``n_total`` the global pool size.
    """

    def __init__(self, pool, excluded=None, device=None, row_base: int = 0, n_total=None,
                 n_pad=None, gram: str = None):
        torch = _torch()
        self.gram = _gram_kind(gram)
        dev = _require_cuda(device)
        lib = _lib.load()
        if isinstance(pool, torch.Tensor):
            x = pool.to(device=dev, dtype=torch.float32)
        else:
            x = torch.from_numpy(np.ascontiguousarray(np.asarray(pool, dtype=np.float32))).to(dev)
        if x.dim() != 2:
            raise ValueError("pool must be a 2-D [rows, features] array")
        self.x = x.contiguous()
        self.device = dev
        self.n, self.d = int(x.shape[0]), int(x.shape[1])
        self.row_base = int(row_base)
        self.n_total = int(n_total) if n_total is not None else self.n
        self.n_pad = int(lib.dal_pad_rows(self.n)) if n_pad is None else int(n_pad)
        if self.n_pad < self.n or self.n_pad % 512:
            raise ValueError("n_pad must be a multiple of 512 and >= the row count")
        self.d_pad = int(lib.dal_pad_features(self.d))
        self.flags = torch.zeros(self.n, dtype=torch.uint8, device=dev)
        self.excluded = np.zeros(0, dtype=np.int64)
        self.set_excluded(excluded)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self._u = None
        self._split = None
        self._norm64 = None
        self._density = None
        self._colsum_partials = None
        self._colsum = None
        self._density_exact = None
        self._acc_pre = None  # density accumulator already zeroed by the prep kernel
        self._xb = None  # blocked feature-major copy of x (dal_pool_blocked), built by the first warm step
        self.blocked_copy = True  # False: never build it (saves n x d fp32 of HBM; same bits, slower K2)
        self._us_steps = 0  # uncertainty steps taken on this pool (the blocked copy pays off from the second)
        self._ws_clean = {}   # (n, k, cap) -> workspace whose top-k header is zero (dal_dw_step)
        self.gram_events = None  # list -> (start, end) HIP events around each Gram call
        self.residual_events = []  # (start, end) HIP events around each residual call (with gram_events)
        self.forest_events = None  # list -> (start, end) HIP events around each forest-score call
        self.select_events = None  # list -> (start, end) HIP events around each dal_dw_select call
        # bench only: a callable run after an eager (per-kernel timed) density
        # step with the step's inputs -- it times the fused step's selection
        # launch on its own (bench.time_step_select; single GPU, fast level 1)
        self.step_select_probe = None
        # bench: a GPU spin (torch.cuda._sleep cycles) queued before each timed
        # call's start event, so the call's launches are all submitted before
        # the GPU reaches them -- the events then bracket the device span, not
        # the host's submission gaps between a call's kernels
        self.event_lead_cycles = 0
        # bench: each timed call is issued this many times back to back between
        # its two events (identical, idempotent launches; the event pair's own
        # cost -- a marker and cache release per record -- is amortised)
        self.event_repeat = 1
        self.cap_scale = 1  # re-rank candidate capacity multiplier, kept after an overflow
        self.cap_base = None  # initial re-rank capacity override (tests: force the overflow path)
        self.level1_fast = True  # fast top-k level 1 allowed (cleared after an overflow on this pool)
        self.use_graphs = True  # hipGraph replay of warm steps (tests compare with eager steps)
        self._graphs = {}  # warm-step graphs by (T, depth, k, beta, cap, level-1 passes)
        self.last_status = 0     # status word read by the last synchronising select

    def clear_caches(self):
        """Drop normalised rows, density, column sums and the blocked copy
        (forces a cold step)."""
        self._u = self._norm64 = self._density = self._colsum = self._colsum_partials = None
        self._split = self._density_exact = self._xb = None
        self._graphs = {}

    def blocked_pool(self, forest, build: bool = True):
        """The pool's blocked feature-major copy (dal_pool_blocked) when the
        forest is one the blocked score kernel applies to (it then reads only
        the features the forest tests), else None.  Built on first use
        (``build``) on the current stream and kept with the pool's caches:
        the warm steps build it, the cold step keeps the row-major kernel.
        The copy costs another n x d fp32 (2 GB at config 4): it is skipped
        (the row-major kernel then runs, same bits) when ``blocked_copy`` is
        False or the device lacks that much free memory plus a 1 GiB margin."""
        if self.n == 0 or not self.blocked_copy:
            return None
        lib = _lib.load()
        if not lib.dal_forest_blocked_rows(self.d, forest.n_trees, forest.depth):
            return None
        if self._xb is None and build:
            torch = _torch()
            floats = int(lib.dal_pool_blocked_floats(self.n, self.d))
            free, _ = torch.cuda.mem_get_info(self.device)
            if free < 4 * floats + (1 << 30):
                return None
            xb = torch.empty(floats, dtype=torch.float32, device=self.device)
            call("dal_pool_blocked", _ptr(self.x), self.n, self.d, self.d, _ptr(xb), _stream(self.device))
            self._xb = xb
        return self._xb

    # ------------------------------------------------------------- caches
    def set_excluded(self, excluded):
        """E (global indices): dropped from the density as i and as j
        (density_weighting.py:95-100)."""
        torch = _torch()
        ex = np.unique(np.asarray([] if excluded is None else list(excluded) if isinstance(excluded, range)
                                  else excluded, dtype=np.int64).reshape(-1))
        if ex.size and (ex[0] < 0 or ex[-1] >= self.n_total):
            # the density error bound counts |E| columns: an index outside the
            # pool would make the interval keys (and the exact selection) unsound
            raise ValueError(f"excluded indices must lie in [0, {self.n_total})")
        if np.array_equal(ex, self.excluded) and hasattr(self, "_u"):
            return
        self.excluded = ex
        self.flags.zero_()
        local = ex[(ex >= self.row_base) & (ex < self.row_base + self.n)] - self.row_base
        if local.size:
            self.flags[torch.from_numpy(local).to(self.device)] = DAL_ROW_EXCLUDED
        self._u = self._norm64 = self._density = self._colsum = self._colsum_partials = None
        self._split = self._density_exact = None
        self._graphs = {}

    def n_excluded_global(self) -> int:
        return int(self.excluded.size)

    def norms(self):
        """Canonical fp64 row norms [n]: those of the fused normalise+split
        pass once the Gram operand exists, else from dal_normalize_rows."""
        if self._norm64 is None:
            self.normalized()
        return self._norm64

    def normalized(self):
        """(u [n_pad, d_pad] fp32 with E rows zeroed, norm64 [n] fp64)."""
        if self._u is None:
            torch = _torch()
            if self.n == 0:
                self._u = torch.zeros((self.n_pad, self.d_pad), dtype=torch.float32, device=self.device)
                self._norm64 = torch.zeros(0, dtype=torch.float64, device=self.device)
                return self._u, self._norm64
            self._u = torch.empty((self.n_pad, self.d_pad), dtype=torch.float32, device=self.device)
            self._norm64 = torch.empty(self.n, dtype=torch.float64, device=self.device)
            call("dal_normalize_rows", _ptr(self.x), self.n, self.d, self.d, _ptr(self.flags),
                 self.n_pad, self.d_pad, _ptr(self._u), _ptr(self._norm64), _ptr(self.status),
                 _stream(self.device))
        return self._u, self._norm64

    def gram_operand(self, with_partials: bool = True, acc_zero=None):
        """The density GEMM's operand for this shard's rows: the fp32 unit rows
        (gram "f32") or their two-term fp16 split [n_pad, 2*d_pad] (gram
        "sym", dal_prep_split).  All-gathered as is in the multi-GPU path.
        with_partials: the fused prep also writes the canonical column-sum
        partials (else they are left to colsum_partials()).  acc_zero: an
        int64 [n_pad] density accumulator to zero (by the prep kernel when it
        runs here, else by a fill)."""
        if self.gram == "f32":
            u, _ = self.normalized()
            if acc_zero is not None:
                acc_zero.zero_()
            return u
        zeroed = False
        if self._split is None:
            torch = _torch()
            self._split = torch.empty((self.n_pad, 2 * self.d_pad), dtype=torch.int16, device=self.device)
            if self._u is not None:
                call("dal_split_f16", _ptr(self._u), self.n_pad, self.d_pad, self.d_pad, _ptr(self._split),
                     _stream(self.device))
            elif self.n == 0:  # an empty shard (more GPUs than row granules)
                self._split.zero_()
                if self._norm64 is None:
                    self._norm64 = torch.zeros(0, dtype=torch.float64, device=self.device)
            else:  # fused: the fp32 unit rows never reach HBM; canonical partials on the way
                norm64 = torch.empty(self.n, dtype=torch.float64, device=self.device)
                chunks = (self.n + DAL_CANON_CHUNK - 1) // DAL_CANON_CHUNK
                parts = None
                if self._colsum_partials is None and with_partials:
                    parts = torch.empty((chunks, self.d), dtype=torch.float64, device=self.device)
                call("dal_prep_split", _ptr(self.x), self.n, self.d, self.d, _ptr(self.flags),
                     self.n_pad, self.d_pad, _ptr(self._split), _ptr(norm64),
                     0 if parts is None else _ptr(parts), 0 if acc_zero is None else _ptr(acc_zero),
                     _ptr(self.status), _stream(self.device))
                zeroed = True
                if self._norm64 is None:
                    self._norm64 = norm64
                if parts is not None:
                    self._colsum_partials = parts
        if acc_zero is not None and not zeroed:
            acc_zero.zero_()
        return self._split

    def colsum_partials(self):
        """Canonical fp64 column-sum partials of this shard ([chunks, d])."""
        if self._colsum_partials is None:
            torch = _torch()
            norm64 = self.norms()
            chunks = (self.n + DAL_CANON_CHUNK - 1) // DAL_CANON_CHUNK
            self._colsum_partials = torch.empty((chunks, self.d), dtype=torch.float64, device=self.device)
            call("dal_canon_colsum_partials", _ptr(self.x), self.n, self.d, self.d, _ptr(norm64),
                 _ptr(self.flags), _ptr(self._colsum_partials), _stream(self.device))
        return self._colsum_partials

    def colsum(self, partials=None):
        """s = sum_{j not in E} u_j in the canonical fp64 order."""
        if partials is not None:
            torch = _torch()
            s = torch.empty(self.d, dtype=torch.float64, device=self.device)
            call("dal_canon_colsum_reduce", _ptr(partials), int(partials.shape[0]), self.d, _ptr(s),
                 _stream(self.device))
            return s
        if self._colsum is None:
            self._colsum = self.colsum(self.colsum_partials())
        return self._colsum

    def density_fixed(self, u_cols=None, n_cols_pad=None):
        """int64 fixed-point Gram row-sums (value * 2^32) of this shard's rows
        against every column of ``u_cols`` (default: this pool)."""
        if self._density is None or u_cols is not None:
            torch = _torch()
            op = self.gram_operand()
            if self.gram == "sym" and u_cols is not None:
                raise ValueError("gram 'sym' over a gathered operand: use ShardedSelector")
            if self.gram == "sym" and (self.row_base or self.n_total != self.n):
                raise ValueError("gram 'sym' on a shard: use ShardedSelector")
            if u_cols is None and self._acc_pre is not None:
                acc, self._acc_pre = self._acc_pre, None  # zeroed by the prep kernel
            else:
                acc = torch.zeros(self.n_pad, dtype=torch.int64, device=self.device)
            cols = op if u_cols is None else u_cols
            ncp = self.n_pad if n_cols_pad is None else int(n_cols_pad)
            self.gram_accumulate(acc, cols, ncp)
            if self.gram == "sym":
                self.gram_residual(acc, op)
            if u_cols is not None:
                return acc
            self._density = acc
        return self._density

    def nb_active(self) -> int:
        """Global count of 256-row blocks (pad512(N_total) / 256)."""
        return (self.n_total + 511) // 512 * 2

    def gram_accumulate(self, acc, cols, n_cols_pad: int, grid_blocks: int = 0, col_row0: int = 0,
                        skip=None):
        """acc += fixed-point row sums of this shard's rows against the first
        ``n_cols_pad`` (a multiple of 512) rows of ``cols`` (a Gram operand of
        the pool's kind), whose first row is global row ``col_row0``.  Exact:
        any column split adds up to the same bits.

        gram "sym": acc is indexed by GLOBAL row (length >= nb_active * 256)
        and receives ONLY the row sums of this shard's own rows over the
        super-block pairs they take; the column sums of every pair come in
        closed form from gram_residual, so no collective follows (ABI v8).
        ``skip`` = (row0, row1), global column rows (multiples of 256) left
        out (gram "sym" only: already accumulated)."""
        torch = _torch()
        op = self.gram_operand()
        ev = None
        if self.gram_events is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        if self.gram == "sym":
            nb = self.nb_active()
            j_lo = col_row0 // 256
            j_hi = min(j_lo + int(n_cols_pad) // 256, nb)
            s_lo, s_hi = (0, 0) if skip is None else (skip[0] // 256, skip[1] // 256)
            if j_hi > j_lo and self.row_base // 256 < nb:
                call("dal_gram_rowsum_sym_skip", _ptr(op), self.row_base // 256, self.n_pad // 256,
                     _ptr(cols), j_lo, j_lo, j_hi, s_lo, s_hi, nb, self.d_pad, _ptr(acc), int(grid_blocks),
                     _stream(self.device))
        elif skip is not None:
            raise ValueError("a skipped column range needs gram 'sym'")
        else:
            call("dal_gram_rowsum", _ptr(op), self.n_pad, _ptr(cols), int(n_cols_pad), self.d_pad,
                 self.d_pad, _ptr(acc), int(grid_blocks), _stream(self.device))
        if ev is not None:
            ev[1].record()
            self.gram_events.append(ev)
        return acc

    def gram_residual(self, acc, ops):
        """Complete the compensated symmetric Gram (gram "sym"): add the exact
        remainder of the H-only A side for this shard's rows into acc (global
        row index).  ``ops``: the operand of EVERY active row (this pool's, or
        the gathered one on several GPUs)."""
        torch = _torch()
        lib = _lib.load()
        nb = self.nb_active()
        rb0, nrb = self.row_base // 256, self.n_pad // 256
        if rb0 >= nb or self.n == 0:
            return acc
        wsb = int(lib.dal_gram_sym_residual_workspace_bytes(nb, nrb, self.d_pad))
        ws, wsp = workspace(wsb, self.device)
        ev = None
        if self.gram_events is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        call("dal_gram_sym_residual", _ptr(ops), nb, rb0, nrb, self.d_pad, _ptr(acc), wsp, wsb,
             _stream(self.device))
        if ev is not None:
            ev[1].record()
            self.residual_events.append(ev)
        del ws
        return acc

    def events_off(self) -> bool:
        """No per-launch HIP-event timing requested (the graph path has none)."""
        return self.forest_events is None and self.select_events is None and self.gram_events is None

    def set_density_fixed(self, acc):
        self._density = acc

    def density_exact(self, colsum=None):
        """Separable canonical fp64 density of this shard's rows (NaN for E):
        the exact identity sum_j <u_i,u_j> = <u_i, s>, O(N*D), bit-identical to
        the oracle.  ``colsum`` = the global s (multi-GPU); default this pool's."""
        if self._density_exact is None or colsum is not None:
            torch = _torch()
            norm64 = self.norms()
            s = self.colsum() if colsum is None else colsum
            d = torch.empty(self.n, dtype=torch.float64, device=self.device)
            call("dal_density_separable", _ptr(self.x), self.n, self.d, self.d, _ptr(norm64), _ptr(s),
                 _ptr(self.flags), _ptr(d), _stream(self.device))
            if colsum is not None:
                return d
            self._density_exact = d
        return self._density_exact

    def density(self, mode: str = "gram"):
        """fp64 density d[n] (NaN for rows in E): the MFMA Gram row-sum / 2^32
        (mode "gram", the reference's algorithm) or the exact separable form
        (mode "separable")."""
        torch = _torch()
        if mode == "separable":
            return self.density_exact()
        if mode != "gram":
            raise ValueError(f"density mode must be 'gram' or 'separable', not {mode!r}")
        d = self.density_fixed()[: self.n].to(torch.float64) * (1.0 / DAL_FIXED_SCALE)
        ex = (self.flags & DAL_ROW_EXCLUDED).bool()
        return torch.where(ex, torch.full_like(d, float("nan")), d)

    # ------------------------------------------------------------ helpers
    def row_flags(self, unlabeled_idx):
        """EXCLUDED bits | CANDIDATE for the (global) unlabeled indices of this
        shard, built on the device (no host round trip).  Returns (flags,
        unlabeled indices, count of unlabeled indices)."""
        unl = _as_index(unlabeled_idx, self.device)
        flags = self.flags.clone()
        call("dal_mark_rows", _ptr(unl), int(unl.shape[0]), self.row_base, self.n,
             DAL_ROW_CANDIDATE, _ptr(flags), _stream(self.device))
        return flags, unl, int(unl.shape[0])

    def local_positions(self, unl):
        """Rows of this shard for global indices ``unl`` (single GPU: all of them)."""
        if self.row_base == 0 and self.n == self.n_total:
            return unl
        loc = unl - self.row_base
        return loc[(loc >= 0) & (loc < self.n)]

    def check_status(self, st=None):
        """Raise on the device status word (``st``: a value already read)."""
        if st is None:
            st = int(self.status.item())
        if st & DAL_FLAG_ZERO_NORM:
            raise ValueError("pool contains a zero-norm row: cosine similarity is undefined "
                             "(the reference would propagate NaN into every density)")
        if st & DAL_FLAG_CAND_OVERFLOW:
            raise _lib.DalError("density re-rank candidate set exceeded DAL_SORT_CAP_PAYLOAD")
        if st & DAL_FLAG_SAMPLE_MISS:
            raise _lib.DalError("fast top-k level 1 overflowed and was not re-run")


GRAM_KINDS = ("sym", "f32")


def _gram_kind(gram) -> str:
    """Density GEMM kernel: "sym" (default; fp16 MFMA on the two-term split,
    each symmetric block pair once, H-only taker side + exact closed-form
    remainder) or "f32" (fp32 MFMA on the unit rows, every pair: the
    plain-precision reference kernel, chosen per pool by the caller).  Both
    are within their rigorous bound of the canonical density and give the
    same (bit-exact) selection."""
    g = "sym" if gram is None else gram
    if g not in GRAM_KINDS:
        raise ValueError(f"gram must be one of {GRAM_KINDS}, not {g!r}")
    return g


def gram_products(state: PoolState) -> int:
    """fp16 MFMA products per feature pair of the pool's Gram kernel (bench
    roofline: executed vs algorithmic flops)."""
    return 2 if state.gram == "sym" else 1


def _as_index(idx, device):
    torch = _torch()
    if isinstance(idx, torch.Tensor):
        if idx.dtype is torch.int64 and idx.is_cuda and idx.get_device() == device.index and idx.is_contiguous():
            return idx  # already a device index list (the AL loop's steady state)
        return idx.to(device=device, dtype=torch.int64).contiguous()
    return torch.from_numpy(np.asarray(idx, dtype=np.int64).reshape(-1)).to(device)


def as_pool_state(pool, excluded=None, device=None) -> PoolState:
    if isinstance(pool, PoolState):
        if excluded is not None:
            pool.set_excluded(excluded)
        return pool
    return PoolState(pool, excluded=excluded, device=device)


_LUT_CACHE = {}


_SIDE_STREAMS = {}


def _side_stream(device):
    """One auxiliary HIP stream per device (created once)."""
    torch = _torch()
    key = str(device)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return _SIDE_STREAMS[key]


def device_lut(strategy: str, n_trees: int, device):
    """fp64 LUT on the device, uploaded once per (strategy, T, device)."""
    torch = _torch()
    key = (strategy, int(n_trees), str(device))
    if key not in _LUT_CACHE:
        _LUT_CACHE[key] = torch.from_numpy(make_lut(strategy, n_trees)).to(device)
    return _LUT_CACHE[key]


def forest_score(state: PoolState, forest: Forest, lut_dev, flags, order: int, density=None,
                 density_err: float = 0.0, beta: float = 1.0, want_hi: bool = False,
                 density_kind=None, xb=None):
    """Launch dal_forest_score (dal_forest_score_blocked over ``xb``, the
    pool's blocked copy) over the shard; returns (votes, scores, keys, keys_hi)."""
    torch = _torch()
    forest.check_features(state.d)
    inner, leaf = forest.device(state.device)
    n = state.n
    votes = torch.empty(n, dtype=torch.int32, device=state.device)
    scores = torch.empty(n, dtype=torch.float64, device=state.device)
    keys = torch.empty(n, dtype=torch.int64, device=state.device)
    keys_hi = torch.empty(n, dtype=torch.int64, device=state.device) if want_hi else None
    if density is None:
        kind = DAL_DENSITY_NONE
    elif density_kind is not None:
        kind = density_kind
    else:
        kind = DAL_DENSITY_EXACT if density.dtype == torch.float64 else DAL_DENSITY_FIXED
    ev = None
    if state.forest_events is not None:  # bench: K2 launch timing on the launch stream
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        if state.event_lead_cycles:
            torch.cuda._sleep(state.event_lead_cycles)
        ev[0].record()
    args = (n, state.d, state.d, _ptr(inner), _ptr(leaf), forest.n_trees, forest.depth, _ptr(lut_dev),
            0 if density is None else _ptr(density), kind, float(density_err), _ptr(flags), float(beta), int(order),
            _ptr(votes), _ptr(scores), _ptr(keys), 0 if keys_hi is None else _ptr(keys_hi), _stream(state.device))
    for _ in range(state.event_repeat if ev is not None else 1):
        if xb is None:
            call("dal_forest_score", _ptr(state.x), *args)
        else:
            call("dal_forest_score_blocked", _ptr(state.x), _ptr(xb), _fprep(forest, state, xb), *args)
    if ev is not None:
        ev[1].record()
        state.forest_events.append(ev)
    return votes, scores, keys, keys_hi


def _fprep(forest: Forest, state: PoolState, xb) -> int:
    """Address of the forest prepared for the blocked kernel (0 without xb)."""
    if xb is None:
        return 0
    p = forest.blocked_prep(state.device, state.d)
    return 0 if p is None else _ptr(p)


def topk_keys(keys, k: int, idx_base: int = 0):
    """k smallest keys (ties -> lower index): (indices int64 [k], keys [k])."""
    torch = _torch()
    lib = _lib.load()
    n = int(keys.shape[0])
    ws = torch.empty(int(lib.dal_topk_workspace_bytes(n, k)) + 256, dtype=torch.uint8,
                     device=keys.device)
    wsp = (_ptr(ws) + 255) // 256 * 256
    out_idx = torch.empty(k, dtype=torch.int64, device=keys.device)
    out_keys = torch.empty(k, dtype=torch.int64, device=keys.device)
    call("dal_topk", _ptr(keys), n, k, int(idx_base), wsp, int(lib.dal_topk_workspace_bytes(n, k)),
         _ptr(out_idx), _ptr(out_keys), _stream(keys.device))
    return out_idx, out_keys


def density_error(state: PoolState) -> float:
    """Bound on |d_gemm - d_canonical| (rigorous; dal_density_error_bound or
    _sym, by the pool's Gram kernel)."""
    n_cols = max(state.n_total - state.n_excluded_global(), 1)
    lib = _lib.load()
    if state.gram == "f32":
        return float(lib.dal_density_error_bound(n_cols))
    return float(lib.dal_density_error_bound_sym_d(n_cols, state.d_pad))


def candidate_cap(n: int, k: int) -> int:
    """Initial re-rank candidate capacity (grown on overflow).  Up to
    DAL_SORT_CAP_PAYLOAD the exact second level is a single one-block sort."""
    return int(min(n, max(4 * k, _lib.DAL_SORT_CAP_PAYLOAD)))


# Fast level 1 of the interval selections (ABI v6): tau = the k-th smallest
# of <= 4096 row groups' minimum keys bounds the candidate search (group
# minima + one launch instead of 6 radix passes + 3 compaction launches);
# 0 selects the exact radix level 1 (after an overflow, per pool).
LEVEL1_PASSES = 1


def level1_passes(state, n: int, k: int, cap: int) -> int:
    if not state.level1_fast or cap > DAL_SORT_CAP_PAYLOAD:
        return 0
    return LEVEL1_PASSES


def workspace(nbytes: int, device):
    """A 256-byte aligned device workspace: (tensor, aligned pointer)."""
    torch = _torch()
    ws = torch.empty(int(nbytes) + 256, dtype=torch.uint8, device=device)
    return ws, (_ptr(ws) + 255) // 256 * 256


def dw_select_local(state: PoolState, flags, votes, keys_lo, keys_hi, lut_dev, k: int,
                    beta: float, colsum, cap_scale: int = 1, sync: bool = True, colsum_ready=None):
    """dal_dw_select on this shard: exact canonical top-k of the shard.  The
    candidate capacity grows (and the step re-runs) on DAL_FLAG_CAND_OVERFLOW.
    colsum_ready: a torch.cuda.Event recorded after ``colsum`` on another
    stream; the library joins it just before the re-rank (its only reader).
    sync=False: no status read here -- the caller checks state.status later
    and re-runs with a larger cap_scale on overflow (multi-GPU path)."""
    torch = _torch()
    lib = _lib.load()
    n = state.n
    norm64 = state.norms()
    if sync:  # single-GPU: start from the capacity a previous overflow grew to
        cap_scale = max(cap_scale, state.cap_scale)
    base = candidate_cap(n, k) if state.cap_base is None else max(int(k), int(state.cap_base))
    cap = int(min(n, base * cap_scale))
    while True:
        passes = level1_passes(state, n, k, cap)
        wsb = int(lib.dal_dw_select_workspace_bytes(n, k, cap))
        ws, wsp = workspace(wsb, state.device)
        out_idx = torch.empty(k, dtype=torch.int64, device=state.device)
        out_scores = torch.empty(k, dtype=torch.float64, device=state.device)
        out_keys = torch.empty(k, dtype=torch.int64, device=state.device)
        ev = None
        if state.select_events is not None:  # bench: K3 timing on the launch stream
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            if state.event_lead_cycles:
                torch.cuda._sleep(state.event_lead_cycles)
            ev[0].record()
        for _ in range(state.event_repeat if ev is not None else 1):
            call("dal_dw_select", _ptr(keys_lo), _ptr(keys_hi), _ptr(votes), _ptr(flags), n, k,
                 state.row_base, _ptr(lut_dev), float(beta), _ptr(state.x), state.d, state.d,
                 _ptr(norm64), _ptr(colsum), cap, passes, wsp, wsb, _ptr(out_idx), _ptr(out_scores),
                 _ptr(out_keys), _ptr(state.status),
                 0 if colsum_ready is None else colsum_ready.cuda_event, _stream(state.device))
        if ev is not None:
            ev[1].record()
            state.select_events.append(ev)
        if not sync:
            return out_idx, out_scores, out_keys
        # the step's one host sync: status word (zero-norm rows, candidate overflow)
        st = int(state.status.item())
        state.last_status = st
        if st & DAL_FLAG_SAMPLE_MISS:  # fast level 1 over capacity: exact level 1 from now on
            state.status.bitwise_and_(~(DAL_FLAG_SAMPLE_MISS | DAL_FLAG_CAND_OVERFLOW))
            state.level1_fast = False
            continue
        if cap >= n or not (st & DAL_FLAG_CAND_OVERFLOW):
            return out_idx, out_scores, out_keys
        state.status.bitwise_and_(~DAL_FLAG_CAND_OVERFLOW)
        cap = min(n, cap * 4)
        state.cap_scale *= 4  # later steps (same pool, same score spread) start here


def dw_step_local(state: PoolState, forest: Forest, flags, dens, lut_dev, k: int, beta: float, colsum,
                  colsum_ready=None, cap_scale: int = None, sync: bool = True, xb=None):
    """dal_dw_step on this pool or shard: votes, scores and interval keys
    of every row, then the exact canonical top-k -- one C call with fused
    launches (the fast level 1; ``xb``: the pool's blocked copy for the score
    kernel).  Same retries as dw_select_local.
    Returns (votes, scores, indices, selected scores); sync=False (the
    multi-GPU path: the caller reads the status word after the merge and
    re-runs with a larger ``cap_scale``) also returns the selected keys."""
    torch = _torch()
    lib = _lib.load()
    n = state.n
    forest.check_features(state.d)
    inner, leaf = forest.device(state.device)
    norm64 = state.norms()
    derr = float(density_error(state))
    dev = state.device
    votes = torch.empty(n, dtype=torch.int32, device=dev)
    scores = torch.empty(n, dtype=torch.float64, device=dev)
    keys_lo = torch.empty(n, dtype=torch.int64, device=dev)
    keys_hi = torch.empty(n, dtype=torch.int64, device=dev)
    base = candidate_cap(n, k) if state.cap_base is None else max(int(k), int(state.cap_base))
    cap = int(min(n, base * (state.cap_scale if cap_scale is None else cap_scale)))
    while True:
        passes = level1_passes(state, n, k, cap)
        wsb = int(lib.dal_dw_step_workspace_bytes(n, k, cap))
        # one workspace per (n, k, cap), zeroed once: DAL_STEP_WS_CLEAN leaves
        # its header zero after every call (no zeroing launch per step)
        key = (n, k, cap)
        if key not in state._ws_clean:
            ws, wsp = workspace(wsb, dev)
            ws.zero_()
            state._ws_clean[key] = (ws, wsp)
        ws, wsp = state._ws_clean[key]
        out_idx = torch.empty(k, dtype=torch.int64, device=dev)
        out_scores = torch.empty(k, dtype=torch.float64, device=dev)
        out_keys = None if sync else torch.empty(k, dtype=torch.int64, device=dev)
        try:
            call("dal_dw_step", _ptr(state.x), 0 if xb is None else _ptr(xb), _fprep(forest, state, xb), n,
                 state.d, state.d, _ptr(inner),
                 _ptr(leaf), forest.n_trees, forest.depth, _ptr(lut_dev), _ptr(dens), derr, _ptr(flags),
                 float(beta), state.row_base,
                 _ptr(norm64), _ptr(colsum), k, cap, passes, DAL_STEP_WS_CLEAN, wsp, wsb, _ptr(votes),
                 _ptr(scores), _ptr(keys_lo), _ptr(keys_hi), _ptr(out_idx), _ptr(out_scores),
                 0 if out_keys is None else _ptr(out_keys), _ptr(state.status),
                 0 if colsum_ready is None else colsum_ready.cuda_event, _stream(dev))
        except _lib.DalError:
            # a call that failed after queueing part of the step may leave the
            # level-1 header dirty: never reuse this workspace as "clean"
            state._ws_clean.pop(key, None)
            raise
        if not sync:
            return votes, scores, out_idx, out_scores, out_keys
        st = int(state.status.item())  # the step's one host sync
        state.last_status = st
        if st & DAL_FLAG_SAMPLE_MISS:  # fast level 1 over capacity: exact level 1 from now on
            state.status.bitwise_and_(~(DAL_FLAG_SAMPLE_MISS | DAL_FLAG_CAND_OVERFLOW))
            state.level1_fast = False
            continue
        if cap >= n or not (st & DAL_FLAG_CAND_OVERFLOW):
            return votes, scores, out_idx, out_scores
        state.status.bitwise_and_(~DAL_FLAG_CAND_OVERFLOW)
        cap = min(n, cap * 4)
        state.cap_scale *= 4


def sort_pairs(keys, idx, k: int, payload=None):
    """Sort (key, idx) pairs (with an optional fp64 payload) and keep k."""
    torch = _torch()
    n = int(keys.shape[0])
    k = min(k, n)
    out_keys = torch.empty(k, dtype=torch.int64, device=keys.device)
    out_idx = torch.empty(k, dtype=torch.int64, device=keys.device)
    out_pay = torch.empty(k, dtype=torch.float64, device=keys.device) if payload is not None else None
    call("dal_sort_pairs", _ptr(keys), _ptr(idx), 0 if payload is None else _ptr(payload), n, k,
         _ptr(out_keys), _ptr(out_idx), 0 if out_pay is None else _ptr(out_pay), _stream(keys.device))
    return out_keys, out_idx, out_pay


# ---------------------------------------------------------------- steps --
def uncertainty_blocked(state: PoolState, forest: Forest):
    """The blocked pool copy for an uncertainty step (scores only, no
    density: every step is alike): built from the pool's second step on --
    the one-off copy costs about five row-major score launches (2M x 256:
    0.92 ms vs 0.2 ms saved per launch), so a pool scored once keeps the
    row-major kernel."""
    state._us_steps += 1
    return state.blocked_pool(forest, build=state._us_steps > 1)


def uncertainty_step(state: PoolState, unlabeled_idx, forest: Forest, k: int,
                     strategy: str = "least_confidence") -> Selection:
    """One iteration of uncertainty_sampling.py:85-112 on the GPU."""
    flags, unl, n_cand = state.row_flags(unlabeled_idx)
    if n_cand == 0:
        raise ValueError("unlabeled set is empty (the reference loop breaks here)")
    kk = min(int(k), n_cand)
    loc = state.local_positions(unl)
    order = DAL_ASCENDING if ASCENDING[strategy] else DAL_DESCENDING
    lut_dev = device_lut(strategy, forest.n_trees, state.device)
    votes, scores, keys, _ = forest_score(state, forest, lut_dev, flags, order,
                                          xb=uncertainty_blocked(state, forest))
    idx, _ = topk_keys(keys, kk, state.row_base)
    sel_scores = scores[idx - state.row_base]
    state.check_status()
    return Selection(scores=(scores, loc), indices=idx, selected_scores=sel_scores, votes=(votes, loc))


def density_step(state: PoolState, unlabeled_idx, forest: Forest, k: int, beta: float = 1.0,
                 density_fixed=None, mode: str = "gram") -> Selection:
    """One iteration of density_weighting.py:133-176 on the GPU:
    score = ent[v] * d^beta, descending; exact canonical selection.

    mode "gram": density from the fused MFMA Gram row-sum (the reference's
    N^2 algorithm) with an exact fp64 re-rank of the boundary candidates;
    mode "separable": density from the exact O(N*D) identity (scores are then
    canonical fp64 for every row and the top-k needs no re-rank)."""
    if mode == "separable":
        return _density_step_separable(state, unlabeled_idx, forest, k, beta)
    if mode != "gram":
        raise ValueError(f"density mode must be 'gram' or 'separable', not {mode!r}")
    unl = _as_index(unlabeled_idx, state.device)
    if int(unl.shape[0]) == 0:
        raise ValueError("unlabeled set is empty (the reference loop breaks here)")
    if (state.use_graphs and density_fixed is None and state._density is not None and state._colsum is not None
            and state.row_base == 0 and state.n == state.n_total and state.events_off()):
        return _density_step_graph(state, unl, forest, min(int(k), int(unl.shape[0])), beta)
    # the density GEMM goes to the GPU first; the host prepares the rest while it runs
    colsum_ready = None
    # warm (density cached): the score kernel reads the pool's blocked copy
    # (built by the first warm step); the cold step keeps the row-major kernel
    xb = state.blocked_pool(forest) if state._density is not None or density_fixed is not None else None
    if density_fixed is None and state._density is None and state._colsum is None and state.n:
        # cold step: the canonical column sum (only the exact re-rank needs it)
        # runs on a side stream AFTER the Gram, beside the vote / score chain
        # (beside the Gram itself it would slow the persistent Gram blocks)
        torch = _torch()
        # the fused prep also writes the canonical column-sum partials (the side
        # stream below then only reduces them: 56 us less per config-2 step than
        # computing them after the Gram) and zeroes the density accumulator
        acc = torch.empty(state.n_pad, dtype=torch.int64, device=state.device)
        state.gram_operand(with_partials=True, acc_zero=acc)
        state._acc_pre = acc
        dens = state.density_fixed()
        main = torch.cuda.current_stream(state.device)
        side = _side_stream(state.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            cs = state.colsum()
            colsum_ready = torch.cuda.Event()
            colsum_ready.record(side)
        cs.record_stream(main)
    else:
        dens = state.density_fixed() if density_fixed is None else density_fixed
    flags, unl, n_cand = state.row_flags(unl)
    kk = min(int(k), n_cand)
    loc = state.local_positions(unl)
    lut_dev = device_lut("entropy", forest.n_trees, state.device)
    if (state.forest_events is None and state.select_events is None and state.row_base == 0
            and state.n == state.n_total):
        # one C call, fused launches (the per-kernel timing path below keeps K2 / K3 apart)
        votes, scores, idx, sel_scores = dw_step_local(state, forest, flags, dens, lut_dev, kk, beta,
                                                       state.colsum(), colsum_ready, xb=xb)
        state.check_status(state.last_status)
        return Selection(scores=(scores, loc), indices=idx, selected_scores=sel_scores, votes=(votes, loc))
    votes, scores, keys_lo, keys_hi = forest_score(
        state, forest, lut_dev, flags, DAL_DESCENDING, density=dens,
        density_err=density_error(state), beta=beta, want_hi=True, xb=xb)
    # the main stream joins the column sum inside the call, just before the re-rank
    idx, sel_scores, _ = dw_select_local(state, flags, votes, keys_lo, keys_hi, lut_dev, kk, beta,
                                         state.colsum(), colsum_ready=colsum_ready)
    state.check_status(state.last_status)  # the word dw_select_local read (no second sync)
    if state.select_events is not None and state.step_select_probe is not None and state.level1_fast:
        state.step_select_probe(state, forest, flags, dens, lut_dev, kk, beta, xb)
    return Selection(scores=(scores, loc), indices=idx, selected_scores=sel_scores, votes=(votes, loc))


class WarmStepGraph:
    """One warm density-weighted step (density cached -- the reference's
    per-iteration path, density_weighting.py:133-176) as a libdal plan
    (dal_dw_plan_create): dal_dw_step -- forest votes + score + interval
    keys, the candidate search, the exact fp64 re-rank and the final sort,
    fused into 5 launches -- captured once as a hipGraph over static device
    buffers.  Per step ONE C call (dal_dw_plan_run) rebuilds the row flags
    from the pool's base flags and the unlabeled list, replays the graph,
    copies the selection out and reads the status word.  A different forest
    is copied into the static heap arrays first."""

    def __init__(self, state: PoolState, forest: Forest, k: int, beta: float, cap: int, passes: int,
                 colsum=None, packed=None):
        """colsum: the canonical column sum to re-rank against (default the
        pool's own; a shard passes the global one).  packed: an int64 [3k+1]
        row receiving (selected keys | indices | score bits | status) -- the
        multi-GPU top-k all-gather row -- instead of the plan's own buffers."""
        import ctypes

        torch = _torch()
        dev = state.device
        n = state.n
        self.state, self.k, self.cap, self.passes = state, int(k), int(cap), int(passes)
        forest.check_features(state.d)
        inner, leaf = forest.device(dev)
        self.inner, self.leaf = inner.clone(), leaf.clone()
        self.forest_ref = forest
        self.n_trees, self.depth = forest.n_trees, forest.depth
        self.flags = state.flags.clone()
        self.lut = device_lut("entropy", forest.n_trees, dev)
        self.votes = torch.empty(n, dtype=torch.int32, device=dev)
        self.scores = torch.empty(n, dtype=torch.float64, device=dev)
        self.keys_lo = torch.empty(n, dtype=torch.int64, device=dev)
        self.keys_hi = torch.empty(n, dtype=torch.int64, device=dev)
        self.packed = packed
        if packed is None:
            # selected indices and scores side by side: one copy hands them out
            self.out_pair = torch.empty(2 * k, dtype=torch.int64, device=dev)
            self.out_keys = torch.empty(k, dtype=torch.int64, device=dev)
            status = state.status
        else:
            if packed.dtype != torch.int64 or tuple(packed.shape) != (3 * k + 1,) or not packed.is_contiguous():
                raise ValueError("packed must be a contiguous int64 [3k+1] tensor")
            packed.zero_()  # the status slot's upper half stays zero
            self.out_keys, self.out_pair = packed[:k], packed[k:3 * k]
            status = packed[3 * k:].view(torch.int32)[:1]  # low half of the last word (little endian)
        self.status = status
        self._last = None  # weak reference to the Selection that still reads votes / scores
        lib = _lib.load()
        self.wsb = int(lib.dal_dw_step_workspace_bytes(n, k, cap))
        self.ws, self.wsp = workspace(self.wsb, dev)
        xb = state.blocked_pool(forest)  # the score kernel reads the pool's blocked copy when it applies
        # the forest prepared for the blocked kernel, in a static buffer the
        # plan reads at its captured address (re-prepared when the forest changes)
        self.fprep = None
        if xb is not None:
            nb = int(lib.dal_forest_prep_bytes(state.d, self.n_trees, self.depth))
            if nb:
                self.fprep = torch.empty(nb, dtype=torch.uint8, device=dev)
                self._prepare()
        self._keep = (state.density_fixed(), state.colsum() if colsum is None else colsum, state.norms(),
                      state.flags, state.x, xb)
        dens, colsum, norm64 = self._keep[:3]
        plan = ctypes.c_void_p()
        call("dal_dw_plan_create", _ptr(state.x), 0 if xb is None else _ptr(xb),
             0 if self.fprep is None else _ptr(self.fprep), n, state.d, state.d,
             _ptr(self.inner), _ptr(self.leaf),
             self.n_trees, self.depth, _ptr(self.lut), _ptr(dens), float(density_error(state)), _ptr(state.flags),
             _ptr(self.flags), float(beta), state.row_base, _ptr(norm64), _ptr(colsum), k, cap, passes, self.wsp,
             self.wsb, _ptr(self.votes), _ptr(self.scores), _ptr(self.keys_lo), _ptr(self.keys_hi),
             _ptr(self.out_pair), _ptr(self.out_keys), _ptr(status), _stream(dev), ctypes.byref(plan))
        self.plan = plan
        self._status = ctypes.c_int32()
        self._status_ref = ctypes.byref(self._status)
        self._run = lib.dal_dw_plan_run
        self._finalizer = weakref.finalize(self, lib.dal_dw_plan_destroy, plan)

    def _prepare(self):
        """dal_forest_prepare of the plan's static forest copy into its static
        prepared buffer (stream-ordered before the next replay)."""
        if self.fprep is not None:
            call("dal_forest_prepare", _ptr(self.inner), _ptr(self.leaf), self.n_trees, self.depth, self.state.d,
                 _ptr(self.fprep), int(self.fprep.shape[0]), _stream(self.state.device))

    def run(self, forest: Forest, unl):
        """Refresh the inputs, replay, read the status: returns (votes,
        scores, selected indices, selected scores, status).  votes / scores
        are the plan's buffers, valid until the next replay (copy-on-write:
        the previous step's Selection is materialised before they are
        reused); the selection lands in fresh tensors."""
        torch = _torch()
        prev = self._last() if self._last is not None else None
        if prev is not None:
            prev._detach()
        dev = self.state.device
        if forest is not self.forest_ref:
            forest.check_features(self.state.d)
            inner, leaf = forest.device(dev)
            self.inner.copy_(inner)
            self.leaf.copy_(leaf)
            self._prepare()
            self.forest_ref = forest
        idx = torch.empty(self.k, dtype=torch.int64, device=dev)
        sc = torch.empty(self.k, dtype=torch.float64, device=dev)
        rc = self._run(self.plan, unl.data_ptr(), unl.shape[0], idx.data_ptr(), sc.data_ptr(), self._status_ref,
                       _raw_stream(dev))
        if rc:
            _lib.check(rc, "dal_dw_plan_run")
        return self.votes, self.scores, idx, sc, self._status.value

    def launch(self, forest: Forest, unl):
        """Refresh and replay on the current stream WITHOUT waiting (the
        outputs land in ``packed``); the caller reads the status later."""
        if forest is not self.forest_ref:
            forest.check_features(self.state.d)
            inner, leaf = forest.device(self.state.device)
            self.inner.copy_(inner)
            self.leaf.copy_(leaf)
            self._prepare()
            self.forest_ref = forest
        call("dal_dw_plan_launch", self.plan, unl.data_ptr(), int(unl.shape[0]), _raw_stream(self.state.device))


def _density_step_graph(state: PoolState, unl, forest: Forest, kk: int, beta: float) -> Selection:
    """Warm density step through a cached WarmStepGraph (same selection as
    the eager path; a level-1 or re-rank capacity overflow rebuilds the plan
    with the exact level 1 / a larger capacity and replays)."""
    n = state.n
    loc = state.local_positions(unl)
    while True:
        base = candidate_cap(n, kk) if state.cap_base is None else max(int(kk), int(state.cap_base))
        cap = int(min(n, base * state.cap_scale))
        passes = level1_passes(state, n, kk, cap)
        key = (forest.n_trees, forest.depth, kk, float(beta), cap, passes)
        g = state._graphs.get(key)
        if g is None:
            g = state._graphs[key] = WarmStepGraph(state, forest, kk, beta, cap, passes)
        try:
            votes, scores, idx, sel_scores, st = g.run(forest, unl)
        except _lib.DalError:
            # a failed replay may leave the plan's workspace header dirty: rebuild next time
            state._graphs.pop(key, None)
            raise
        state.last_status = st
        if st & DAL_FLAG_SAMPLE_MISS:
            state.status.bitwise_and_(~(DAL_FLAG_SAMPLE_MISS | DAL_FLAG_CAND_OVERFLOW))
            state.level1_fast = False
            continue
        if (st & DAL_FLAG_CAND_OVERFLOW) and cap < n:
            state.status.bitwise_and_(~DAL_FLAG_CAND_OVERFLOW)
            state.cap_scale *= 4
            continue
        state.check_status(st)
        sel = Selection(scores=(scores, loc), indices=idx, selected_scores=sel_scores, votes=(votes, loc))
        g._last = weakref.ref(sel)
        return sel


def torch_float64():
    return _torch().float64


def _density_step_separable(state: PoolState, unlabeled_idx, forest: Forest, k: int,
                            beta: float) -> Selection:
    flags, unl, n_cand = state.row_flags(unlabeled_idx)
    if n_cand == 0:
        raise ValueError("unlabeled set is empty (the reference loop breaks here)")
    kk = min(int(k), n_cand)
    loc = state.local_positions(unl)
    lut_dev = device_lut("entropy", forest.n_trees, state.device)
    votes, scores, keys, _ = forest_score(state, forest, lut_dev, flags, DAL_DESCENDING,
                                          density=state.density_exact(), beta=beta)
    idx, _ = topk_keys(keys, kk, state.row_base)
    sel_scores = scores[idx - state.row_base]
    state.check_status()
    return Selection(scores=(scores, loc), indices=idx, selected_scores=sel_scores, votes=(votes, loc))
