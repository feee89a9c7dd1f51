"""Density-weighted selection with beta != 1 (score = entropy x density^beta,
density_weighting.py:33 declares beta; the reference leaves it at 1).  The
score kernels take pow out of line for beta != 1 (forest.hip,
density_pow_general), so this covers that call path: the cold step (Gram
density), the warm plan replay over the blocked pool copy, and the separable
density, each against the oracle's np.power scores.  pow is not required to
round identically in the two libms, so scores are compared to 1e-14 relative
and the selection must be the oracle's."""
import numpy as np
import pytest

from oracle import dal_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("beta", [0.5, 2.0])
@pytest.mark.parametrize("n,d,trees", [(6_000, 64, 10), (5_000, 30, 100)])
def test_density_select_beta(cuda, beta, n, d, trees):
    import torch

    from dal import density_weighting as dw
    from dal.engine import PoolState
    from dal.forest import Forest

    k = 25
    X = O.synthetic_pool(n, d, seed=n + trees)
    E = np.arange(10)
    of = O.synthetic_forest(trees, 4, d, seed=3)
    F = Forest.synthetic(trees, 4, d, seed=3)
    unl = np.arange(10, n)
    _, ref_idx, ref_sc = O.density_select(X, unl, of, k, beta, E)
    st = PoolState(X, excluded=E, device=cuda)
    unl_dev = torch.from_numpy(unl).to(cuda)
    for step in range(3):  # cold, first warm (blocked copy built), warm plan replay
        sel = dw.select(st, unl_dev, F, k, beta=beta)
        got = sel.indices.cpu().numpy()
        assert np.array_equal(got, ref_idx), step
        sc = sel.selected_scores.cpu().numpy()
        assert np.allclose(sc, ref_sc, rtol=1e-14, atol=0.0), step
    sep = dw.select(PoolState(X, excluded=E, device=cuda), unl_dev, F, k, beta=beta, mode="separable")
    assert np.array_equal(sep.indices.cpu().numpy(), ref_idx)
