"""The AL loop driver on the GPU path reproduces the oracle-driven loop
iteration by iteration: with scikit-learn training (same seeds -> same
forests) and with the GPU trainer (dal.random_forest vs oracle/rf_oracle.py on
the same bagging draws -> same trees, same test accuracy, same selections)."""
import numpy as np
import pytest

from conftest import load_golden
from dal import loop
from oracle import dal_oracle as O
from oracle import rf_oracle as R
from test_loop import oracle_select

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("strategy", ["uncertainty", "density"])
@pytest.mark.parametrize("name", ["checkerboard2x2.npz", "rotated_checkerboard2x2.npz"])
def test_gpu_loop_matches_oracle_loop(cuda, strategy, name):
    g = load_golden(name)
    X, y = g["X"], g["y"]
    ref = loop.run_loop(X, y, X, y, strategy=strategy, window_size=10, max_iterations=6,
                        select_fn=oracle_select, trainer="sklearn")
    got = loop.run_loop(X, y, X, y, strategy=strategy, window_size=10, max_iterations=6,
                        device=cuda, trainer="sklearn")
    assert got.log == ref.log
    for a, b in zip(got.labeled_history, ref.labeled_history):
        assert np.array_equal(a, b)


class _OracleModel:
    def __init__(self, forest, n_trees):
        self.forest, self.n_trees = forest, n_trees

    def predict(self, X):
        return (2 * O.votes(self.forest, X) > self.n_trees).astype(np.int64)


def _oracle_trainer(X, y, T, seed):
    from dal.random_forest import bagging_inputs

    w, s = bagging_inputs(X.shape[0], X.shape[1], T, 4, seed)
    _, sf, st, lc = R.train_classifier(X, y.astype(np.int64), w, s)
    return _OracleModel(R.heap_forest(sf, st, lc), T)


def _oracle_select_heap(strategy, X, unlabeled, model, k):
    if strategy == "uncertainty":
        return O.uncertainty_select(X, unlabeled, model.forest, k)[1]
    return O.density_select(X, unlabeled, model.forest, k, 1.0, np.arange(10))[1]


@pytest.mark.parametrize("strategy", ["uncertainty", "density"])
@pytest.mark.parametrize("name", ["checkerboard2x2.npz", "checkerboard4x4.npz"])
def test_gpu_trainer_loop_matches_oracle_trainer_loop(cuda, strategy, name):
    g = load_golden(name)
    X, y = g["X"], g["y"]
    ref = loop.run_loop(X, y, X, y, strategy=strategy, window_size=10, max_iterations=8,
                        select_fn=_oracle_select_heap, trainer=_oracle_trainer)
    got = loop.run_loop(X, y, X, y, strategy=strategy, window_size=10, max_iterations=8,
                        device=cuda, trainer="gpu")
    assert got.log == ref.log  # includes the per-iteration test accuracy
    for a, b in zip(got.labeled_history, ref.labeled_history):
        assert np.array_equal(a, b)
