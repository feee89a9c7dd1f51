"""Pin the CPU oracle (oracle/dal_oracle.py) against the reference's own
known answers and the committed golden fixtures.  CPU only."""
import json
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_forest, load_golden
from oracle import dal_oracle as O


def test_entropy_lut_matches_reference_log_kat():
    """density_weighting.py:148 values printed by the reference itself
    (final_thesis/results/striatum_distDW_window_10_samples_5000.txt)."""
    kat = json.load(open(os.path.join(GOLDEN, "kat_dw_log_T10.json")))
    ent = O.lut_entropy(10)
    finite = [repr(float(x)) for x in ent if not math.isnan(x)]
    # every value the reference printed is one of our table entries, bit for bit
    for v in kat["values_repr"]:
        assert v in finite, v
    # and the table's v=0 entry is the reference's -0.0 (sign included)
    assert repr(float(ent[0])) == "-0.0"
    assert math.isnan(ent[10])
    # v=1 pins the log(x)/log(2) evaluation (numpy's log2 is one ulp off)
    assert repr(float(ent[1])) == "0.13680278410054497"


def test_reference_log_topk_lists_are_descending():
    """The (idx, score) lists the reference printed (density_weighting.py:170)
    are sorted descending under our comparator (-0.0 ties allowed)."""
    kat = json.load(open(os.path.join(GOLDEN, "kat_dw_log_T10.json")))
    assert len(kat["topk_lists"]) >= 10
    for item in kat["topk_lists"]:
        sc = [float(s) for _, s in item["pairs"]]
        assert all(a >= b for a, b in zip(sc, sc[1:])), item["line"]


@pytest.mark.parametrize("T", [10, 50, 100])
def test_lut_golden(T):
    g = load_golden(f"lut_T{T}.npz")
    assert np.array_equal(O.lut_least_confidence(T), g["lc"])
    assert np.array_equal(O.lut_margin(T), g["mg"])
    assert np.array_equal(O.lut_entropy(T), g["ent"], equal_nan=True)


def test_lc_fp64_asymmetric_pairs_t100():
    """The LC score breaks symmetry in fp64: v=41 vs 59."""
    lc = O.lut_least_confidence(100)
    assert repr(float(lc[41])) == "0.09000000000000008"
    assert repr(float(lc[59])) == "0.08999999999999997"
    asym = sum(1 for v in range(50) if lc[v] != lc[100 - v])
    assert asym == 8


GOLDEN_POOLS = ["synthetic_512x64_T10.npz", "synthetic_4096x256_T10.npz",
                "synthetic_1500x30_T100.npz"]


@pytest.mark.parametrize("name", GOLDEN_POOLS)
def test_synthetic_golden_reproduces(name):
    g = load_golden(name)
    f = golden_forest(g)
    X = g["X"]
    assert np.array_equal(O.votes(f, X), g["votes"])
    d = O.density_canonical(X, g["excluded"])
    assert np.array_equal(d, g["density"], equal_nan=True)
    # separable canonical == full fp64 Gram row-sum (the reference algorithm)
    dg = O.density_gram(X, g["excluded"])
    ok = ~np.isnan(dg)
    assert np.allclose(d[ok], dg[ok], rtol=1e-12, atol=1e-9)
    for strat in O.STRATEGIES:
        sc, si, ss = O.uncertainty_select(X, g["unlabeled"], f, 10, strat)
        assert np.array_equal(si, g[f"us_{strat}_k10_idx"])
    sc, si, ss = O.density_select(X, g["unlabeled"], f, 100, 1.0, g["excluded"])
    assert np.array_equal(si, g["dw_k100_idx"])
    assert np.array_equal(ss, g["dw_k100_scores"])


def test_synthetic_forest_matches_heap_draws():
    """The oracle's synthetic forest and the product's Forest.synthetic draw
    identically (same config inputs for bench and tests)."""
    from dal.forest import Forest

    f = O.synthetic_forest(5, 4, 64, seed=1)
    F = Forest.synthetic(5, 4, 64, seed=1)
    X = O.synthetic_pool(300, 64, seed=5)
    v = O.votes(f, X)
    # walk the product's heap layout on the host (test-side reference walk)
    from test_forest_format import heap_votes

    assert np.array_equal(heap_votes(F, X), v)


def test_checkerboard_goldens_have_tie_groups():
    g = load_golden("checkerboard2x2.npz")
    # iteration 1 (10 labeled rows) exercises the heavy-tie path
    v = g["it1_votes"][g["it1_unlabeled"]]
    assert len(np.unique(v)) < 11


def test_select_topk_canonical_rules():
    sc = np.array([0.5, -0.0, 0.0, np.nan, 0.5, 0.1])
    idx = np.arange(6) + 100
    si, ss = O.select_topk(sc, idx, 6, ascending=True)
    assert list(si) == [101, 102, 105, 100, 104, 103]  # -0 == +0 -> index order; NaN last
    si, ss = O.select_topk(sc, idx, 6, ascending=False)
    assert list(si) == [100, 104, 105, 101, 102, 103]


def test_density_excluded_rows_are_nan_and_dropped():
    X = O.synthetic_pool(64, 8, seed=2)
    d = O.density_canonical(X, [0, 5])
    assert np.isnan(d[0]) and np.isnan(d[5])
    U = O.l2_normalize(X)
    keep = np.ones(64, bool)
    keep[[0, 5]] = False
    ref = (U @ U[keep].T).sum(axis=1)
    assert np.allclose(d[keep], ref[keep], rtol=1e-13)


def test_zero_norm_row_rejected():
    X = np.ones((4, 3), np.float32)
    X[2] = 0
    with pytest.raises(ValueError):
        O.l2_normalize(X)
