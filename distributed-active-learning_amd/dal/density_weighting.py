"""Density-weighted uncertainty query step -- drop-in for final_thesis/density_weighting.py.

Reference pipeline:
  proximity matrix  density_weighting.py:58-75  rows L2-normalised (:66), S = U.U^T
                    via BlockMatrix.multiply (:73), N^2 entries pulled to Python (:74-75)
  L0 exclusion      :89-100   entries with i or j in the initial window are dropped once
  per iteration     :136-145  T per-tree predicts + vote sum
                    :148      e = -(1-v/T) log2(1-v/T)
                    :157-161  d_i = sum of the row's remaining S entries (includes j = i)
                    :166-172  score = e * d, descending sortBy, take(window_size)
Here: a fused MFMA Gram row-sum -- fp16 MFMA on a two-term (hi/lo) fp16
split of the unit rows, each symmetric block pair once, plus an exact
closed-form remainder, accumulated in int64 fixed point (S never exists; the density is cached
per pool because the reference's is constant across iterations), a fused
forest + score kernel, and a device top-k whose boundary candidates are
re-ranked in canonical fp64 so the selected set is bit-exact.
``beta`` (declared at :33, unused by the reference) weights d^beta.
"""
from __future__ import annotations

from .engine import PoolState, Selection, as_pool_state, density_step
from .forest import Forest


def information_density(pool, excluded_idx=None, device=None, mode: str = "gram"):
    """d_i = sum_{j not in E} cos(x_i, x_j) for every row (fp64, NaN for i in E).

    excluded_idx  E; the reference uses L0 = range(window_size).
    mode          "gram": fused compensated fp16-split MFMA Gram row-sum (the
                  reference's N^2 algorithm, fp32-class: within
                  dal_density_error_bound_sym of canonical);
                  "separable": exact O(N*D) identity, canonical fp64 bits.
    """
    state = as_pool_state(pool, excluded=excluded_idx, device=device)
    d = state.density(mode)
    state.check_status()
    return d


L0 = "L0"  # excluded_idx default: the reference's initial labeled window


def select(pool, unlabeled_idx, forest: Forest, k: int, beta: float = 1.0, excluded_idx=L0,
           density=None, device=None, mode: str = "gram", window_size=None) -> Selection:
    """Score every unlabeled row by entropy x density^beta and select the top k.

    excluded_idx  rows dropped from the density as i and as j.  Default "L0":
                  the reference's initial labeled window range(window_size)
                  (density_weighting.py:89,95-100); for a PoolState the default
                  keeps the state's own excluded set.  None or [] excludes
                  nothing.
    window_size   the reference's window (L0 = range(window_size)).  Omitted,
                  it is k -- the script takes window_size rows per iteration
                  (:172) -- unless k may be a batch clamped to a short
                  unlabeled set (k >= |unlabeled|), where L0 is ambiguous and
                  window_size must be given.
    density       optional int64 fixed-point density from a previous call
                  (PoolState.density_fixed()); by default the pool's cached one
    mode          "gram" (default, the reference's algorithm on MFMA) or
                  "separable" (exact O(N*D) identity; same selection)
    """
    if isinstance(excluded_idx, str):
        if excluded_idx != L0:
            raise ValueError(f"excluded_idx must be index-like, None or {L0!r}")
        if isinstance(pool, PoolState):
            excluded_idx = None
        else:
            if window_size is None:
                n_unl = len(unlabeled_idx) if hasattr(unlabeled_idx, "__len__") else None
                if n_unl is not None and int(k) >= n_unl:
                    raise ValueError("k >= the unlabeled count: k may be a clamped batch, so L0 = "
                                     "range(window_size) is ambiguous -- pass window_size (or excluded_idx)")
                window_size = k
            excluded_idx = range(int(window_size))
    elif excluded_idx is None and isinstance(pool, PoolState):
        excluded_idx = []
    state = as_pool_state(pool, excluded=excluded_idx, device=device)
    return density_step(state, unlabeled_idx, forest, k, beta=beta, density_fixed=density, mode=mode)


__all__ = ["information_density", "select", "PoolState", "Selection"]
