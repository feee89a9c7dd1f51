"""Uncertainty sampling query step -- drop-in for final_thesis/uncertainty_sampling.py.

The reference's loop body (uncertainty_sampling.py:85-112) runs T Spark jobs of
``DecisionTreeModel(tree).predict`` over the unlabeled pool (:88-93), sums the
hard votes per row (:96-97), scores ``abs(0.5 - (1 - v/T))`` (:98), sorts
ascending (:106) and takes ``window_size`` rows (:109).  Here that is one
fused HIP kernel (votes + fp64 LUT score + sort key) and a device top-k.
Scores are attached to their own rows (the intended alignment of
lal_direct_mllib_implementation/classes/active_learner.py:160-183; the script's
positional re-key at :100-104 mis-aligns rows when Spark shuffles).
Ties (frequent: only T+1 distinct scores) go to the lower pool index.
"""
from __future__ import annotations

from .engine import PoolState, Selection, as_pool_state, uncertainty_step
from .forest import Forest
from .luts import STRATEGIES


def select(pool, unlabeled_idx, forest: Forest, k: int, strategy: str = "least_confidence",
           device=None) -> Selection:
    """Score every unlabeled row and select the k most uncertain.

    pool           [N, D] fp32 (numpy or torch; or a PoolState to reuse caches)
    unlabeled_idx  global row indices of the unlabeled set
    forest         dal.forest.Forest (from_sklearn / from_nodes / synthetic)
    k              batch size (``window_size``; clamped to the unlabeled count)
    strategy       "least_confidence" (reference), "margin" or "entropy"
    Returns Selection(scores[U], indices[k], selected_scores[k], votes[U]).
    """
    if strategy not in STRATEGIES:
        raise ValueError(f"strategy must be one of {STRATEGIES}")
    state = as_pool_state(pool, device=device)
    return uncertainty_step(state, unlabeled_idx, forest, k, strategy)


__all__ = ["select", "PoolState", "Selection"]
