"""Cosine Gram products -- drop-in for final_thesis/cosine_similarity.py.

The reference normalises every row (:28), builds ``U.multiply(UT)`` through
IndexedRowMatrix -> CoordinateMatrix -> BlockMatrix (:29-42) and reads the
N x N entries (:44-45).  ``cosine_entries`` returns that matrix (fp32 MFMA,
small N); ``cosine_rowsum`` is the fused row-sum the density path uses, which
never materialises it.
"""
from __future__ import annotations

from . import _lib
from .engine import _ptr, _stream, as_pool_state


def cosine_entries(pool, device=None):
    """S[i][j] = cos(x_i, x_j) for all i, j (fp32, [N, N], diagonal included)."""
    import torch

    state = as_pool_state(pool, device=device)
    u, _ = state.normalized()
    n_pad32 = (state.n + 31) // 32 * 32
    out = torch.empty((n_pad32, n_pad32), dtype=torch.float32, device=state.device)
    _lib.call("dal_gram_entries", _ptr(u), n_pad32, state.d_pad, state.d_pad, _ptr(out),
              _stream(state.device))
    state.check_status()
    return out[: state.n, : state.n]


def cosine_rowsum(pool, excluded_idx=None, device=None):
    """sum_{j not in E} S[i][j] per row (fp64; NaN for i in E)."""
    from .density_weighting import information_density

    return information_density(pool, excluded_idx, device=device)


__all__ = ["cosine_entries", "cosine_rowsum"]
