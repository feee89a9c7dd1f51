"""AL loop driver + text ingest (dal.loop): host logic on CPU with the
oracle as the selection step; the GPU run of the same loop is in
test_gpu_loop.py."""
import numpy as np
import pytest

from conftest import load_golden
from dal import loop
from oracle import dal_oracle as O


def oracle_select(strategy, X, unlabeled, rf, k):
    of = O.forest_from_sklearn(rf)
    if strategy == "uncertainty":
        return O.uncertainty_select(X, unlabeled, of, k)[1]
    E = np.arange(10)
    return O.density_select(X, unlabeled, of, k, 1.0, E)[1]


def test_load_labeled_text(tmp_path):
    p = tmp_path / "pool.txt"
    p.write_text("1 2 3 -1\n4 5 6 1\n\n7 8 9 -1\n0.5 0.25 1 0\n")
    X, y = loop.load_labeled_text(str(p))
    assert X.dtype == np.float32 and X.shape == (4, 3)
    assert list(y) == [0, 1, 0, 1]  # reference mapping: -1 -> 0, anything else -> 1
    X2, y2 = loop.load_labeled_text(str(p), n_samples=2, label_map="as_is")
    assert X2.shape == (2, 3) and list(y2) == [-1, 1]


@pytest.mark.parametrize("strategy", ["uncertainty", "density", "random"])
def test_loop_runs_to_exhaustion_with_reference_log(strategy):
    g = load_golden("checkerboard2x2.npz")
    X, y = g["X"][:120], g["y"][:120]
    res = loop.run_loop(X, y, X, y, strategy=strategy, window_size=10,
                        select_fn=oracle_select, trainer="sklearn")
    assert res.log[0] == "labeled =  10  unlabeled =  110"
    assert res.log[-1] == "labeled =  120  unlabeled =  0"
    assert res.log[2].startswith("labeled =  20")
    assert res.log[1].startswith("Iteration  1  -- accu =  ")
    chosen = np.concatenate(res.labeled_history)
    assert sorted(chosen.tolist()) == list(range(10, 120))  # every row labeled once
    assert len(res.accuracy) == 11


def test_dw_l0_default_ambiguous_batch_raises_before_gpu():
    """k >= |unlabeled| may be a clamped batch: L0 = range(window_size) cannot
    be inferred from k, so select() asks for window_size (no GPU touched)."""
    from dal import density_weighting as dw

    X = np.random.default_rng(0).random((40, 4))
    with pytest.raises(ValueError, match="window_size"):
        dw.select(X, np.arange(35, 40), None, 5)
