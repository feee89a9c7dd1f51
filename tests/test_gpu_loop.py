"""The AL loop driver on the GPU path reproduces the oracle-driven loop
iteration by iteration (same sklearn seeds -> same forests -> same selections)."""
import numpy as np
import pytest

from conftest import load_golden
from dal import loop
from test_loop import oracle_select

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("strategy", ["uncertainty", "density"])
@pytest.mark.parametrize("name", ["checkerboard2x2.npz", "rotated_checkerboard2x2.npz"])
def test_gpu_loop_matches_oracle_loop(cuda, strategy, name):
    g = load_golden(name)
    X, y = g["X"], g["y"]
    ref = loop.run_loop(X, y, X, y, strategy=strategy, window_size=10, max_iterations=6,
                        select_fn=oracle_select)
    got = loop.run_loop(X, y, X, y, strategy=strategy, window_size=10, max_iterations=6,
                        device=cuda)
    assert got.log == ref.log
    for a, b in zip(got.labeled_history, ref.labeled_history):
        assert np.array_equal(a, b)
