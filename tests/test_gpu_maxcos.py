"""Max-cosine / diversity selection (similarity.py restated for BASELINE
config 5): bf16 MFMA kernel vs the canonical fp64 oracle."""
import numpy as np
import pytest

from oracle import dal_oracle as O

pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("n,d,m", [(3000, 128, 300), (2500, 64, 1024), (1800, 256, 130), (700, 128, 1)])
def test_max_cosine_within_bound(cuda, n, d, m):
    from dal import _lib
    from dal import similarity as sim

    X = O.bf16_round(O.synthetic_pool(n, d, seed=n + d))
    L = np.arange(0, n, max(1, n // m))[:m]
    got, arg = sim.max_cosine(X, L, device=cuda)
    got, arg = _np(got), _np(arg)
    ref, ref_arg = O.max_cosine_canonical(X, L)
    bound = _lib.load().dal_maxcos_error_bound(d)
    assert np.abs(got - ref).max() <= bound
    assert np.allclose(got[L], 1.0, atol=bound)  # labeled rows match themselves
    assert np.array_equal(arg, ref_arg)  # canonical arg-max, first l on ties


def test_max_cosine_signed_data(cuda):
    from dal import _lib
    from dal import similarity as sim

    X = O.bf16_round(O.synthetic_pool(2000, 128, seed=5, dist="normal"))
    L = np.arange(100, 612)
    got, arg = sim.max_cosine(X, L, device=cuda)
    ref, ref_arg = O.max_cosine_canonical(X, L)
    assert np.abs(_np(got) - ref).max() <= _lib.load().dal_maxcos_error_bound(128)
    assert np.array_equal(_np(arg), ref_arg)


@pytest.mark.parametrize("d", [64, 128, 256])
def test_max_cosine_argmax_duplicate_labeled_rows(cuda, d):
    """Duplicated labeled rows (and labeled rows equal up to a positive scale)
    tie exactly: the arg-max is the FIRST position l, as in the canonical
    fp64 oracle (similarity.py:34-38 restated; SURVEY §8(b) max_cosine)."""
    from dal import _lib
    from dal import similarity as sim

    n = 3000
    X = O.bf16_round(O.synthetic_pool(n, d, seed=11 + d))
    X[1000:1010] = X[5]           # pool rows equal to a labeled row
    L = np.concatenate([np.arange(0, 200), [5, 5, 7, 1005], np.arange(200, 300)])
    X[7] = X[3] * 2.0             # same direction as row 3 (exact in bf16)
    got, arg = sim.max_cosine(X, L, device=cuda)
    ref, ref_arg = O.max_cosine_canonical(X, L)
    assert np.abs(_np(got) - ref).max() <= _lib.load().dal_maxcos_error_bound(d)
    assert np.array_equal(_np(arg), ref_arg)
    assert (ref_arg[1000:1010] == 5).all()  # first of the duplicated positions


@pytest.mark.parametrize("n,d,m,k", [(4000, 128, 256, 50), (3000, 64, 700, 200), (2000, 256, 64, 1)])
def test_diversity_select_bit_exact(cuda, n, d, m, k):
    from dal import similarity as sim

    X = O.bf16_round(O.synthetic_pool(n, d, seed=7 * n))
    X[500:520] = X[600]  # duplicate rows -> exact ties, resolved by index
    L = np.arange(m)
    cand = np.arange(m, n)
    sel = sim.diversity_select(X, L, k, candidates=cand, device=cuda)
    ref_idx, ref_sc = O.diversity_select_canonical(X, L, k, candidates=cand)
    assert np.array_equal(_np(sel.indices), ref_idx)
    assert np.array_equal(_np(sel.selected_scores), ref_sc)


def test_diversity_select_scale(cuda):
    """30k x 128 pool, 1,024 labeled rows, k = 1000 (config-5 shape, scaled)."""
    from dal import similarity as sim

    n, d, m, k = 30000, 128, 1024, 1000
    X = O.bf16_round(O.synthetic_pool(n, d, seed=0))
    L = np.arange(m)
    cand = np.arange(m, n)
    sel = sim.diversity_select(X, L, k, candidates=cand, device=cuda)
    ref_idx, ref_sc = O.diversity_select_canonical(X, L, k, candidates=cand)
    assert np.array_equal(_np(sel.indices), ref_idx)
    assert np.array_equal(_np(sel.selected_scores), ref_sc)


@pytest.mark.parametrize("case", ["bucket_overflow", "foreign_candidates"])
def test_diversity_select_fallbacks(cuda, case):
    """The fast level 1 overflowing its 4,096 slots (5,000 identical
    least-similar rows: DAL_FLAG_SAMPLE_MISS, exact re-run), and candidate
    lists holding indices outside the pool (filtered after the status read,
    then re-selected with the true count)."""
    from dal import similarity as sim

    n, d, m, k = 12000, 64, 256, 100
    X = O.bf16_round(O.synthetic_pool(n, d, seed=11))
    L = np.arange(m)
    cand = np.arange(m, n)
    if case == "bucket_overflow":
        far = np.zeros(d, dtype=np.float32)
        far[0] = 1.0  # a corner of the positive orthant: every copy has the same, smallest max-cosine
        X[3000:8000] = O.bf16_round(far[None, :])
    else:
        cand = np.concatenate([cand, np.arange(n, n + 500)])  # not rows of this pool
    sel = sim.diversity_select(X, L, k, candidates=cand, device=cuda)
    ref_idx, ref_sc = O.diversity_select_canonical(X, L, k, candidates=cand[cand < n])
    assert np.array_equal(_np(sel.indices), ref_idx)
    assert np.array_equal(_np(sel.selected_scores), ref_sc)
    if case == "bucket_overflow":
        assert (ref_idx == np.arange(3000, 3100)).all()  # ties -> lower index
