"""Pairwise column similarities -- drop-in for final_thesis/similarity.py.

The reference transposes the normalised pool so that points become columns
(:34-37) and calls ``RowMatrix.columnSimilarities()`` (:38): the exact cosine
of every pair i < j (threshold 0, no diagonal).  Returned here as COO arrays
(i, j, value), the fields of the reference's MatrixEntry records.
"""
from __future__ import annotations

from .cosine_similarity import cosine_entries


def column_similarities(pool, device=None):
    """(i, j, cos(x_i, x_j)) for every pair i < j, row-major order."""
    import torch

    S = cosine_entries(pool, device=device)
    n = S.shape[0]
    ij = torch.triu_indices(n, n, offset=1, device=S.device)
    return ij[0], ij[1], S[ij[0], ij[1]]


# ---------------------------------------------------------------------------
# Batch-mode diversity (BASELINE config 5): max-cosine to a labeled set
# ---------------------------------------------------------------------------
def _bf16_pool(pool, device):
    import numpy as np
    import torch

    from .engine import _require_cuda

    dev = _require_cuda(device)
    if isinstance(pool, torch.Tensor):
        x = pool.to(device=dev)
    else:
        x = torch.from_numpy(np.ascontiguousarray(np.asarray(pool, dtype=np.float32))).to(dev)
    if x.dtype != torch.bfloat16:
        x = x.to(torch.float32).to(torch.bfloat16)  # round to nearest even
    if x.dim() != 2 or x.shape[1] not in (64, 128, 256):
        raise ValueError("bf16 max-cosine needs a [rows, 64|128|256] pool")
    return x.contiguous(), dev


class LabeledSet:
    """The labeled rows as the kernels' B operands: bf16 [m_pad, d] (padding
    rows carry 1/||x|| = NaN, ignored by the max) with fp32 1/||x|| for the
    arg-max kernel, the folded fp16 table 2^15 x/||x|| for the max-only
    kernel (``unit16``, built on first use), and the canonical fp64 unit rows
    (feature-major) for the exact re-rank."""

    def __init__(self, rows_bf16, device):
        import torch

        from . import _lib
        from .engine import _ptr, _stream

        lib = _lib.load()
        m, d = int(rows_bf16.shape[0]), int(rows_bf16.shape[1])
        g = int(lib.dal_maxcos_label_rows_granule(d))
        m_pad = -(-m // g) * g
        self.m, self.d, self.m_pad = m, d, m_pad
        self.rows = torch.zeros((m_pad, d), dtype=torch.bfloat16, device=device)
        self.rows[:m] = rows_bf16
        self.status = torch.zeros(1, dtype=torch.int32, device=device)
        self.inv = torch.empty(m_pad, dtype=torch.float32, device=device)
        _lib.call("dal_inv_norms_bf16", _ptr(self.rows), m, m_pad, d, d, _ptr(self.inv),
                  _ptr(self.status), _stream(device))
        # canonical fp64 unit rows, feature-major [d][m] (the re-rank reads
        # them coalesced across labeled rows)
        self.unit64_t = torch.empty((d, m), dtype=torch.float64, device=device)
        _lib.call("dal_canon_unit_rows_bf16", _ptr(self.rows), m, d, d, 1, _ptr(self.unit64_t),
                  _stream(device))
        self.device = device
        self._unit16 = None

    @property
    def unit16(self):
        """fp16 [m_pad, d] = 2^15 x_l / ||x_l|| (canonical fp64 norm, one
        rounding; padding rows repeat row 0) -- dal_max_cosine_unit's B."""
        if self._unit16 is None:
            import torch

            from . import _lib
            from .engine import _ptr, _stream

            u = torch.empty((self.m_pad, self.d), dtype=torch.float16, device=self.device)
            _lib.call("dal_unit_rows_f16", _ptr(self.rows), self.m, self.m_pad, self.d, self.d, _ptr(u),
                      _ptr(self.status), _stream(self.device))
            self._unit16 = u
        return self._unit16


def max_cosine(pool, labeled_idx, device=None):
    """(m, arg): m_i = max_{l in labeled} cos(x_i, x_l) for every pool row
    (fp32 [N]; bf16 MFMA with fp32 accumulation, |error| <=
    dal_maxcos_error_bound(d)) and its arg-max (int32 [N], the position l in
    ``labeled_idx``; the canonical fp64 arg-max, first l on ties -- rows whose
    fp32 top two cannot be ordered are re-ranked exactly in fp64).

    Restates similarity.py:34-38 (columnSimilarities of the normalised pool,
    i.e. every pairwise cosine) reduced to the nearest labeled row."""
    import torch

    from . import _lib
    from .engine import _as_index, _ptr, _stream

    x, dev = _bf16_pool(pool, device)
    n, d = int(x.shape[0]), int(x.shape[1])
    lab = LabeledSet(x[_as_index(labeled_idx, dev)], dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    arg = torch.empty(n, dtype=torch.int32, device=dev)
    _lib.call("dal_max_cosine", _ptr(x), n, d, _ptr(lab.rows), lab.m_pad, _ptr(lab.inv), 0,
              _ptr(out), _ptr(arg), _ptr(status), _stream(dev))
    _lib.call("dal_maxcos_argmax_resolve", _ptr(x), n, d, d, _ptr(lab.unit64_t), lab.m, _ptr(arg),
              _stream(dev))
    if int(status.item()) | int(lab.status.item()):
        raise ValueError("zero-norm row: cosine undefined")
    return out, arg


def diversity_select(pool, labeled_idx, k: int, candidates=None, device=None, row_base: int = 0,
                     labeled_rows=None):
    """Select the k candidate rows least similar to the labeled set (smallest
    max-cosine, ties -> lower index), exact against the canonical fp64
    max-cosine.  Returns Selection(scores = fp32 max-cos of the candidates,
    indices [k], selected_scores = canonical fp64 max-cos).

    The fp32 values come from the folded-operand kernel (dal_max_cosine_unit,
    within dal_maxcos_unit_error_bound(d) ~ 2^-11 of the canonical values, about
    1000x the bf16 kernel's (3d + 6) 2^-24): the bound only widens the interval
    keys, the selection stays exact through the fp64 re-rank.  When the
    candidate list overflows on that bound (near-tied pools: duplicates,
    clusters), the values are recomputed once with the tighter dal_max_cosine
    (d = 64 / 128 / 256) before the capacity grows; ``scores`` then carry that
    kernel's precision.

    For a row shard (multi-GPU) pass ``row_base`` (global index of row 0),
    global ``candidates`` and the labeled set as ``labeled_rows`` ([m, d],
    replicated on every rank) instead of ``labeled_idx``."""
    import numpy as np
    import torch

    from . import _lib
    from ._lib import DAL_ASCENDING, DAL_FLAG_CAND_OVERFLOW, DAL_FLAG_SAMPLE_MISS, DAL_ROW_CANDIDATE
    from .engine import LEVEL1_PASSES, Selection, _as_index, _ptr, _stream, candidate_cap, workspace

    lib = _lib.load()
    x, dev = _bf16_pool(pool, device)
    n, d = int(x.shape[0]), int(x.shape[1])
    if labeled_rows is not None:
        lab_rows, _ = _bf16_pool(labeled_rows, dev)
    else:
        lab_rows = x[_as_index(labeled_idx, dev)]
    lab = LabeledSet(lab_rows, dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    mx = torch.empty(n, dtype=torch.float32, device=dev)
    # values only (no arg-max): the folded-operand kernel; its wider bound
    # only widens the interval keys -- the fp64 re-rank keeps the selection exact
    _lib.call("dal_max_cosine_unit", _ptr(x), n, d, _ptr(lab.unit16), lab.m_pad, _ptr(mx), _ptr(status),
              _stream(dev))
    bound = float(lib.dal_maxcos_unit_error_bound(d))
    tight = False  # the values are the folded kernel's until a candidate overflow asks for the tighter ones
    in_range = None  # device count of the candidates inside this shard (read with the status)
    if candidates is None:
        flags = torch.full((n,), DAL_ROW_CANDIDATE, dtype=torch.uint8, device=dev)
        cand = torch.arange(n, device=dev)
        n_cand = n
    else:
        flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        gidx = _as_index(candidates, dev)
        # the marking kernel also counts the candidates inside this shard
        in_range = torch.empty(1, dtype=torch.int32, device=dev)
        _lib.call("dal_mark_rows_count", _ptr(gidx), int(gidx.shape[0]), int(row_base), n, DAL_ROW_CANDIDATE,
                  _ptr(flags), _ptr(in_range), _stream(dev))
        cand = gidx - row_base if row_base else gidx
        # an upper bound until the status read: global candidates of other
        # shards are not ours (filtered below, off the common path)
        n_cand = int(cand.shape[0])
        if n_cand == 0:
            return Selection(scores=mx[cand], indices=torch.empty(0, dtype=torch.int64, device=dev),
                             selected_scores=torch.empty(0, dtype=torch.float64, device=dev))
    kk = min(int(k), n_cand)
    lo = torch.empty(n, dtype=torch.int64, device=dev)
    hi = torch.empty(n, dtype=torch.int64, device=dev)
    _lib.call("dal_interval_keys_f32", _ptr(mx), n, bound, _ptr(flags), DAL_ASCENDING, _ptr(lo), _ptr(hi),
              _stream(dev))
    cap = candidate_cap(n, kk)
    passes = LEVEL1_PASSES if cap <= _lib.DAL_SORT_CAP_PAYLOAD else 0
    while True:
        wsb = int(lib.dal_maxcos_select_workspace_bytes(n, kk, cap))
        ws, wsp = workspace(wsb, dev)
        out_idx = torch.empty(kk, dtype=torch.int64, device=dev)
        out_sc = torch.empty(kk, dtype=torch.float64, device=dev)
        _lib.call("dal_maxcos_select", _ptr(lo), _ptr(hi), n, kk, int(row_base), _ptr(x), d, d,
                  _ptr(lab.unit64_t), lab.m, cap, passes, wsp, wsb, _ptr(out_idx), _ptr(out_sc), 0,
                  _ptr(status), _stream(dev))
        # one host read for the status words (and the shard's candidate count)
        words = [status, lab.status] + ([in_range] if in_range is not None else [])
        vals = torch.cat(words).tolist()
        st = vals[0] | vals[1]
        if st & 1:
            raise ValueError("zero-norm row: cosine undefined")
        if in_range is not None and vals[2] < n_cand:
            # candidates outside this shard: filter and redo with the true count
            # (kk must not exceed it, or key-NONE rows would fill the list)
            cand = cand[(cand >= 0) & (cand < n)]
            n_cand, in_range = int(cand.shape[0]), None
            if n_cand == 0:
                return Selection(scores=mx[cand], indices=torch.empty(0, dtype=torch.int64, device=dev),
                                 selected_scores=torch.empty(0, dtype=torch.float64, device=dev))
            kk = min(int(k), n_cand)
            cap = candidate_cap(n, kk)
            passes = LEVEL1_PASSES if cap <= _lib.DAL_SORT_CAP_PAYLOAD else 0
            status.zero_()
            continue
        if st & DAL_FLAG_SAMPLE_MISS and passes > 0:  # the fast level 1 overflowed: exact level 1 first
            passes = 0
            status.zero_()
            continue
        if not tight and st & DAL_FLAG_CAND_OVERFLOW:
            # the exact level 1 also holds too many rows within the folded
            # kernel's bound of the boundary: the bf16 kernel's values (bound
            # ~1000x tighter) and their keys -- not for a fast-level-1 miss alone
            # (identical rows: a tighter bound cannot separate them)
            tight = True
            status.zero_()
            _lib.call("dal_max_cosine", _ptr(x), n, d, _ptr(lab.rows), lab.m_pad, _ptr(lab.inv), 0, _ptr(mx), 0,
                      _ptr(status), _stream(dev))
            bound = float(lib.dal_maxcos_error_bound(d))
            _lib.call("dal_interval_keys_f32", _ptr(mx), n, bound, _ptr(flags), DAL_ASCENDING, _ptr(lo), _ptr(hi),
                      _stream(dev))
            continue
        if cap >= n or not (st & DAL_FLAG_CAND_OVERFLOW):
            break
        status.zero_()
        cap = min(n, cap * 4)
        passes = 0
    return Selection(scores=mx[cand], indices=out_idx, selected_scores=out_sc)


__all__ = ["column_similarities", "max_cosine", "diversity_select", "LabeledSet"]
