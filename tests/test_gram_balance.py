"""Multi-GPU balance of the symmetric Gram (reference: the
BlockMatrix multiply's block cogroup, density_weighting.py:73).

With P ranks each rank multiplies its shard's 512-row super blocks by every
column block: first its own shard's columns (launch 1, beside the operand
all-gather), then every other column in one launch with its own shard as the
skip range (dal/parallel.py ShardedSelector.exchange_density ->
engine.PoolState.gram_accumulate).  Which (row super block P, 256-column block
J) pairs a launch computes is the kernel's orientation rule,
csrc/gram_sym.hip ``takes()``: P takes J (Q = J / 2) iff Q == P, or Q > P with
P + Q even, or Q < P with P + Q odd, and J outside the skip range.  This file
restates that rule and the two launches' ranges, checks that the ranks
together take every unordered super-block pair exactly once, and bounds the
per-rank pair counts (the work: every pair is the same 512 x 256 x D MFMA
tile) at configs 3 and 4 and P = 2, 4, 8.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-active-learning_amd"))
from dal.parallel import shard_range  # noqa: E402

CONFIGS = {"config3": 284_807, "config4": 2_000_000, "config2": 100_000}


def takes(P, J, skip_lo=0, skip_hi=0):
    """csrc/gram_sym.hip takes(): vectorised over arrays P (rows) x J (columns)."""
    P = np.asarray(P)[:, None]
    J = np.asarray(J)[None, :]
    Q = J >> 1
    t = (Q == P) | ((Q > P) & (((P + Q) & 1) == 0)) | ((Q < P) & (((P + Q) & 1) == 1))
    return t & ~((J >= skip_lo) & (J < skip_hi))


def rank_launches(n, world, rank):
    """The (row super blocks, column blocks, skip) of the rank's Gram launches
    (engine.gram_accumulate's j_lo / j_hi / skip for the two calls of
    exchange_density; live super blocks: P < ns_active)."""
    lo, _, shard = shard_range(n, world, rank)
    nb = (n + 511) // 512 * 2
    ns = nb // 2
    rows = np.arange(lo // 512, min((lo + shard) // 512, ns))
    own = (lo // 256, min(lo // 256 + shard // 256, nb))
    out = [(rows, np.arange(*own), (0, 0))]
    if world > 1:
        out.append((rows, np.arange(0, min(world * shard // 256, nb)), own))
    return out


def pair_counts(n, world):
    nb = (n + 511) // 512 * 2
    cover = np.zeros((nb // 2, nb), dtype=np.int32)
    counts = []
    for r in range(world):
        c = 0
        for rows, cols, (s0, s1) in rank_launches(n, world, r):
            if rows.size == 0 or cols.size == 0:
                continue
            t = takes(rows, cols, s0, s1)
            c += int(t.sum())
            cover[rows[:, None], cols[None, :]] += t.astype(np.int32)
        counts.append(c)
    return np.array(counts), cover


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_every_pair_taken_once(cfg, world):
    n = CONFIGS[cfg]
    _, cover = pair_counts(n, world)
    ns = cover.shape[0]
    # the kernel's rule over all super blocks: each unordered pair {P, Q} once
    # (diagonal: both column blocks of Q = P), i.e. the taken (P, J) grid
    full = takes(np.arange(ns), np.arange(2 * ns)).astype(np.int32)
    assert np.array_equal(cover, full)
    sb = full.reshape(ns, ns, 2).sum(axis=2)
    both = sb + sb.T
    assert np.all(np.diag(sb) == 2)
    off = ~np.eye(ns, dtype=bool)
    assert np.all(both[off] == 2)  # {P, Q} taken by exactly one of P, Q (both of Q's column blocks)


@pytest.mark.parametrize("cfg,world", [(c, w) for c in ("config3", "config4") for w in (2, 4, 8)])
def test_rank_balance(cfg, world):
    """Per-rank pairs: max/min <= 1.02 wherever the shards hold equal super
    blocks up to one; the only larger spread is config 3 at P = 4 / 8, where
    the LAST rank's shard is 3 super blocks short (equal 512-row granule
    shards, the remainder on the last rank): max/min 1.022 / 1.045, but the
    step time is set by the max, which is within 0.6 % of the mean."""
    counts, _ = pair_counts(CONFIGS[cfg], world)
    ratio, over_mean = counts.max() / counts.min(), counts.max() / counts.mean()
    if cfg == "config3" and world >= 4:
        assert counts[:-1].max() == counts[:-1].min()  # only the last rank differs
        assert ratio <= 1.05 and over_mean <= 1.006
    else:
        assert ratio <= 1.02, (counts, ratio)
    # the orientation rule itself is balanced: pairs per row super block
    # differ by at most one column super block across the whole pool
    n = CONFIGS[cfg]
    ns = (n + 511) // 512
    per_sb = takes(np.arange(ns), np.arange(2 * ns)).sum(axis=1)
    assert per_sb.max() - per_sb.min() <= 2
