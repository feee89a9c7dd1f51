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


@pytest.mark.parametrize("n,d,m,k", [(4000, 128, 256, 50), (3000, 64, 700, 200), (2000, 256, 64, 1),
                                     (4500, 64, 1500, 50)])  # m > 1024: the re-rank's fp32 dots per chunk
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


@pytest.mark.parametrize("case", ["bucket_overflow", "foreign_candidates", "near_ties"])
def test_diversity_select_fallbacks(cuda, case):
    """The fast level 1 overflowing its 4,096 slots (5,000 identical
    least-similar rows: DAL_FLAG_SAMPLE_MISS, exact re-run), candidate lists
    holding indices outside the pool (filtered after the status read, then
    re-selected with the true count), and 5,000 distinct near-tied rows (max-cos
    within ~1e-4 of each other: inside the folded kernel's 2^-11 bound, so the
    values are recomputed with the tighter bf16 kernel)."""
    from dal import similarity as sim

    n, d, m, k = 12000, 64, 256, 100
    X = O.bf16_round(O.synthetic_pool(n, d, seed=11))
    L = np.arange(m)
    cand = np.arange(m, n)
    if case == "bucket_overflow":
        far = np.zeros(d, dtype=np.float32)
        far[0] = 1.0  # a corner of the positive orthant: every copy has the same, smallest max-cosine
        X[3000:8000] = O.bf16_round(far[None, :])
    elif case == "near_ties":
        rng = np.random.default_rng(5)
        near = np.zeros((5000, d), dtype=np.float32)
        near[:, 0] = 1.0
        rows = np.arange(5000)
        near[rows, rng.integers(1, d, 5000)] += rng.integers(1, 9, 5000) * 2.0 ** -10
        near[rows, rng.integers(1, d, 5000)] += rng.integers(1, 9, 5000) * 2.0 ** -12
        X[3000:8000] = O.bf16_round(near)
    else:
        cand = np.concatenate([cand, np.arange(n, n + 500)])  # not rows of this pool
    sel = sim.diversity_select(X, L, k, candidates=cand, device=cuda)
    ref_idx, ref_sc = O.diversity_select_canonical(X, L, k, candidates=cand[cand < n])
    assert np.array_equal(_np(sel.indices), ref_idx)
    assert np.array_equal(_np(sel.selected_scores), ref_sc)
    if case == "bucket_overflow":
        assert (ref_idx == np.arange(3000, 3100)).all()  # ties -> lower index


def _unit_max(cuda, X, L):
    import torch

    from dal import _lib
    from dal import similarity as sim

    x, dev = sim._bf16_pool(X, cuda)
    lab = sim.LabeledSet(x[torch.as_tensor(L, device=dev)], dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.empty(x.shape[0], dtype=torch.float32, device=dev)
    _lib.call("dal_max_cosine_unit", x.data_ptr(), x.shape[0], x.shape[1], lab.unit16.data_ptr(), lab.m_pad,
              out.data_ptr(), st.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    return _np(out).astype(np.float64), int(st.item()) | int(lab.status.item())


@pytest.mark.parametrize("n,d,m,dist", [(3000, 128, 300, "uniform"), (2500, 64, 1024, "uniform"),
                                        (1800, 256, 130, "normal"), (700, 128, 1, "normal")])
def test_max_cosine_unit_within_bound(cuda, n, d, m, dist):
    """The folded-operand kernel (fp16 unit labeled rows, power-of-two
    rescaled pool rows): |m_gpu - m_canonical| <= dal_maxcos_unit_error_bound."""
    from dal import _lib

    X = O.bf16_round(O.synthetic_pool(n, d, seed=n + 3 * d, dist=dist))
    L = np.arange(0, n, max(1, n // m))[:m]
    got, st = _unit_max(cuda, X, L)
    ref, _ = O.max_cosine_canonical(X, L)
    bound = _lib.load().dal_maxcos_unit_error_bound(d)
    assert st == 0
    assert np.abs(got - ref).max() <= bound
    assert np.abs(got - ref).max() > 0  # the fp16 operand is not the bf16 one


@pytest.mark.parametrize("d", [64, 128, 256])
def test_max_cosine_unit_dynamic_range(cuda, d):
    """Rows spanning many binades (whole rows scaled by 2^-100 .. 2^100 and
    entries down to 2^-40 of the row maximum, i.e. below the fp16 range after
    the row rescale; labeled rows with entries below fp16's normal range):
    the bound still holds (the rescale is exact, only tiny entries flush)."""
    from dal import _lib

    rng = np.random.default_rng(d)
    n = 2048
    X = rng.standard_normal((n, d)).astype(np.float32)
    X *= np.exp2(rng.integers(-40, 1, size=(n, d))).astype(np.float32)  # entry magnitudes over 40 binades
    X *= np.exp2(rng.integers(-100, 101, size=(n, 1))).astype(np.float32)  # whole-row scales
    X = O.bf16_round(X)
    X[X.any(axis=1) == 0, 0] = 1.0
    L = np.arange(0, n, 7)[:200]
    got, st = _unit_max(cuda, X, L)
    ref, _ = O.max_cosine_canonical(X, L)
    assert st == 0
    assert np.abs(got - ref).max() <= _lib.load().dal_maxcos_unit_error_bound(d)


def test_max_cosine_unit_zero_row_flags(cuda):
    X = O.bf16_round(O.synthetic_pool(600, 64, seed=3))
    X[17] = 0.0
    _, st = _unit_max(cuda, X, np.arange(0, 600, 3))
    assert st & 1
