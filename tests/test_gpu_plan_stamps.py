"""The warm-step plan's 8-bit row stamps (plan.hip: step ids cycle through
1..255, dal_dw_plan_run clears the stamps when they wrap).  A row marked
unlabeled at replay 1 and never listed again must not come back as a
candidate at replay 256, when the step id is 1 again; every replay's
selection must equal the oracle's for its own unlabeled list
(density_weighting.py:109-176, the loop body over a shrinking list)."""
import numpy as np
import pytest

from oracle import dal_oracle as O

pytestmark = pytest.mark.gpu


def test_plan_stamps_wrap(cuda):
    import torch

    from dal import density_weighting as dw
    from dal.engine import PoolState
    from dal.forest import Forest

    n, d, k = 6_000, 32, 20
    X = O.synthetic_pool(n, d, seed=31)
    E = np.arange(10)
    of = O.synthetic_forest(10, 4, d, seed=2)
    F = Forest.synthetic(10, 4, d, seed=2)
    st = PoolState(X, excluded=E, device=cuda)
    full = np.arange(10, n)
    half = np.arange(10, n // 2)
    _, ref_full, _ = O.density_select(X, full, of, k, 1.0, E)
    _, ref_half, ref_half_ss = O.density_select(X, half, of, k, 1.0, E)
    assert not np.isin(ref_full, half).all()  # the full list's top rows are not all in the half
    half_dev = torch.from_numpy(half).to(cuda)
    full_dev = torch.from_numpy(full).to(cuda)
    dw.select(st, full_dev, F, k)  # cold
    for step in range(1, 301):  # warm replays 1..300 (the plan's step ids wrap after 255)
        unl = full_dev if step == 1 else half_dev
        sel = dw.select(st, unl, F, k)
        got = sel.indices.cpu().numpy()
        if step == 1:
            assert np.array_equal(got, ref_full)
        elif step in (2, 254, 255, 256, 257, 300):
            assert np.array_equal(got, ref_half), step
            assert np.array_equal(sel.selected_scores.cpu().numpy(), ref_half_ss), step
        else:
            assert got.max() < n // 2, step
    assert len(st._graphs) == 1  # one plan replayed throughout
