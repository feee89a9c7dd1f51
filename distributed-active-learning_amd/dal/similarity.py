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


__all__ = ["column_similarities"]
