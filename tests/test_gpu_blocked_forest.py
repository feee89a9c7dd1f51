"""K2 over the pool's blocked feature-major copy (ABI v9: dal_pool_blocked +
dal_forest_score_blocked; ABI v10: the forest prepared once by
dal_forest_prepare, checked entry by entry; uncertainty_sampling.py:88-98,
density_weighting.py:136-167).  The blocked kernel reads only the features
the forest tests, so it must give dal_forest_score's votes, scores and keys
bit for bit on every shape the rule admits: ragged tile tails (n not a
multiple of 64, n < 64), forests testing one feature or the last one, ragged
(shallower) trees, uncertainty and both density kinds; the fused step and
the warm plan must select what they select without it; and the engine's warm
steps (which build the copy) must equal the oracle."""
import numpy as np
import pytest

from oracle import dal_oracle as O

pytestmark = pytest.mark.gpu


def _forest_score_pair(cuda, X, F, density_kind, order=None, flags_unl=None):
    import torch

    from dal import _lib, engine
    from dal._lib import call

    n, d = X.shape
    st = engine.PoolState(X, excluded=np.arange(min(10, n)), device=cuda)
    lib = _lib.load()
    assert lib.dal_forest_blocked_rows(d, F.n_trees, F.depth) == 64  # the path under test
    xb = torch.full((int(lib.dal_pool_blocked_floats(n, d)),), float("nan"), dtype=torch.float32, device=cuda)
    S = torch.cuda.current_stream(cuda).cuda_stream
    call("dal_pool_blocked", st.x.data_ptr(), n, d, d, xb.data_ptr(), S)
    # the copy itself: tile-major, feature-major inside a tile, zero tail rows
    t = xb.view(-1, d, 64).permute(0, 2, 1).reshape(-1, d)
    assert torch.equal(t[:n], st.x) and int(t[n:].count_nonzero()) == 0
    unl = np.arange(min(10, n), n) if flags_unl is None else flags_unl
    flags, _, _ = st.row_flags(unl)
    lut = engine.device_lut("entropy" if density_kind else "least_confidence", F.n_trees, cuda)
    dens, kind, derr = None, _lib.DAL_DENSITY_NONE, 0.0
    if density_kind == "fixed":
        dens, kind, derr = st.density_fixed(), _lib.DAL_DENSITY_FIXED, engine.density_error(st)
    elif density_kind == "exact":
        dens, kind = st.density_exact(), _lib.DAL_DENSITY_EXACT
    order = _lib.DAL_DESCENDING if order is None else order
    a = engine.forest_score(st, F, lut, flags, order, density=dens, density_err=derr, want_hi=True,
                            density_kind=kind if dens is not None else None)
    b = engine.forest_score(st, F, lut, flags, order, density=dens, density_err=derr, want_hi=True,
                            density_kind=kind if dens is not None else None, xb=xb)  # prepared forest (ABI v10)
    # the prepared forest itself: header {fu, bad, nodes, fu_max}, the sorted
    # distinct features as the list, every node's feature as its run's byte
    # offset in the LDS tile (slot * 64 rows * 4 B)
    prep = F.blocked_prep(cuda, d)
    assert prep is not None
    hdr = prep[:16].view(torch.int32).cpu().numpy()
    feats = np.unique(F.inner[..., 0])
    nn = F.inner.shape[0] * F.inner.shape[1]
    assert hdr[0] == feats.size and hdr[1] == 0 and hdr[2] == nn and hdr[3] >= feats.size
    pay = prep[16:].cpu().numpy()
    nodes = pay[:nn * 8].view(np.int32).reshape(-1, 2)
    assert np.array_equal(nodes[:, 0], np.searchsorted(feats, F.inner[..., 0].reshape(-1)) * 256)
    assert np.array_equal(nodes[:, 1], F.inner[..., 1].reshape(-1))
    lb = -(-F.leaf.size // 4) * 4
    assert np.array_equal(pay[nn * 8:nn * 8 + F.leaf.size], F.leaf.reshape(-1))
    used = pay[nn * 8 + lb:nn * 8 + lb + 2 * feats.size].view(np.uint16)
    assert np.array_equal(used, feats)
    # the same kernel building its forest per block (fprep = NULL): the same bits
    inner, leaf = F.device(cuda)
    c = [torch.empty_like(t) for t in b]
    P = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
    call("dal_forest_score_blocked", P(st.x), P(xb), 0, n, d, d, P(inner), P(leaf), F.n_trees, F.depth, P(lut),
         P(dens), kind, float(derr), P(flags), 1.0, int(order), *[P(t) for t in c], S)
    _same(b, c)
    return st, a, b


def _same(a, b):
    import torch

    for u, v in zip(a, b):
        if u.dtype == torch.float64:
            u, v = u.view(torch.int64), v.view(torch.int64)
        assert torch.equal(u, v)


@pytest.mark.parametrize("n,d,trees,kind", [(100_003, 256, 10, "fixed"), (5_000, 256, 10, "none"),
                                            (37, 256, 10, "exact"), (64, 96, 4, "fixed"), (20_000, 512, 10, "fixed"),
                                            (12_345, 200, 7, "none"),
                                            (3_001, 256, 100, "fixed")])  # 256 runs: the 8-wave blocks
def test_blocked_forest_bit_identical(cuda, n, d, trees, kind):
    from dal.forest import Forest

    X = O.synthetic_pool(n, d, seed=n % 97)
    F = Forest.synthetic(trees, 4, d, seed=3)
    st, a, b = _forest_score_pair(cuda, X, F, None if kind == "none" else kind)
    _same(a, b)
    if n <= 5_000:  # votes vs the oracle's traversal too
        of = O.synthetic_forest(trees, 4, d, seed=3)
        assert np.array_equal(b[0].cpu().numpy(), O.votes(of, X))


@pytest.mark.parametrize("feature", ["one", "last", "first_and_last"])
def test_blocked_forest_degenerate_feature_sets(cuda, feature):
    """Forests testing one feature (one 256-B run per tile), only the last
    feature (slot 0 is feature d - 1), or the two ends."""
    from dal.forest import Forest

    n, d = 9_001, 256
    X = O.synthetic_pool(n, d, seed=7)
    F = Forest.synthetic(10, 4, d, seed=5)
    inner = F.inner.copy()
    if feature == "one":
        inner[..., 0] = 17
    elif feature == "last":
        inner[..., 0] = d - 1
    else:
        inner[..., 0] = np.where(np.arange(inner.shape[1]) % 2 == 0, 0, d - 1)[None, :]
    G = Forest(inner=inner, leaf=F.leaf.copy(), depth=F.depth)
    _, a, b = _forest_score_pair(cuda, X, G, "fixed")
    _same(a, b)


@pytest.mark.parametrize("d", [30, 33, 64])
@pytest.mark.parametrize("feature", ["random", "first", "last", "ends"])
def test_blocked_forest_small_d_many_nodes(cuda, d, feature):
    """d <= 64 and >= 512 nodes (T = 100): the block setup ORs the feature
    bitmap's one or two words per wave (forest.hip, wave_or) -- every node on
    feature 0, on d - 1 (the second word when d > 32), on the two ends, or the
    synthetic forest's random features."""
    from dal.forest import Forest

    n = 7_001
    X = O.synthetic_pool(n, d, seed=d)
    F = Forest.synthetic(100, 4, d, seed=13)
    inner = F.inner.copy()
    if feature == "first":
        inner[..., 0] = 0
    elif feature == "last":
        inner[..., 0] = d - 1
    elif feature == "ends":
        inner[..., 0] = np.where(np.arange(inner.shape[1]) % 2 == 0, 0, d - 1)[None, :]
    G = Forest(inner=inner, leaf=F.leaf.copy(), depth=F.depth)
    _, a, b = _forest_score_pair(cuda, X, G, "fixed")
    _same(a, b)


def test_blocked_forest_ragged_trees(cuda):
    """Ragged trees padded into the depth-2 heap (Forest.from_nodes: padding
    nodes test feature 0 against +inf) through the blocked kernel."""
    from dal.forest import Forest

    rng = np.random.default_rng(11)
    d, T = 64, 5
    feats, thr, left, right, value, roots = [], [], [], [], [], []
    for _ in range(T):  # root -> (leaf, inner -> (leaf, leaf))
        base = len(feats)
        roots.append(base)
        feats += [int(rng.integers(d)), -1, int(rng.integers(d)), -1, -1]
        thr += [float(rng.random()), 0.0, float(rng.random()), 0.0, 0.0]
        left += [base + 1, -1, base + 3, -1, -1]
        right += [base + 2, -1, base + 4, -1, -1]
        value += [0, int(rng.integers(2)), 0, int(rng.integers(2)), int(rng.integers(2))]
    F = Forest.from_nodes(np.array(feats), np.array(thr), np.array(left), np.array(right), np.array(value),
                          np.array(roots))
    X = O.synthetic_pool(3_000, d, seed=2)
    _, a, b = _forest_score_pair(cuda, X, F, "fixed")
    _same(a, b)


def test_dw_step_and_plan_with_blocked_copy(cuda):
    """dal_dw_step with xb (the score kernel's 64-row tiles are the row
    groups' blocks) equals the step without it; the warm plan built with the
    copy replays the same selection."""
    import torch

    from dal import _lib, engine
    from dal._lib import DAL_STEP_WS_CLEAN, call
    from dal.forest import Forest

    n, d, k = 300_000, 256, 100
    X = O.synthetic_pool(n, d, seed=8)
    st = engine.PoolState(X, excluded=np.arange(10), device=cuda)
    unl = np.arange(10, n)
    F = Forest.synthetic(10, 4, d, seed=1)
    dens, colsum, norm64 = st.density_fixed(), st.colsum(), st.norms()
    flags, _, _ = st.row_flags(unl)
    lut = engine.device_lut("entropy", 10, cuda)
    inner, leaf = F.device(cuda)
    lib = _lib.load()
    cap = engine.candidate_cap(n, k)
    wsb = int(lib.dal_dw_step_workspace_bytes(n, k, cap))
    P = lambda t: t.data_ptr()  # noqa: E731
    S = torch.cuda.current_stream(cuda).cuda_stream
    xb = st.blocked_pool(F)
    assert xb is not None
    res = []
    for use in (None, xb):
        ws, wsp = engine.workspace(wsb, cuda)
        ws.zero_()
        outs = [torch.empty(n, dtype=t, device=cuda) for t in (torch.int32, torch.float64, torch.int64, torch.int64)]
        i1 = torch.empty(k, dtype=torch.int64, device=cuda)
        c1 = torch.empty(k, dtype=torch.float64, device=cuda)
        st.status.zero_()
        call("dal_dw_step", P(st.x), 0 if use is None else P(use), 0, n, d, d, P(inner), P(leaf), 10, 4, P(lut),
             P(dens), float(engine.density_error(st)), P(flags), 1.0, 0, P(norm64), P(colsum), k, cap, 1,
             DAL_STEP_WS_CLEAN, wsp, wsb, *[P(t) for t in outs], P(i1), P(c1), 0, P(st.status), 0, S)
        assert int(st.status.item()) == 0
        res.append(outs + [i1, c1])
    _same(res[0], res[1])
    of = O.synthetic_forest(10, 4, d, seed=1)
    _, ref_idx, ref_ss = O.density_select(X, unl, of, k, 1.0, np.arange(10))
    assert np.array_equal(res[1][4].cpu().numpy(), ref_idx)
    # the engine: cold (row-major kernel), then warm plan replays (blocked copy built by the first)
    from dal import density_weighting as dw

    st2 = engine.PoolState(X, excluded=np.arange(10), device=cuda)
    for it in range(3):
        sel = dw.select(st2, unl, F, k)
        assert (st2._xb is not None) == (it > 0)
        assert np.array_equal(sel.indices.cpu().numpy(), ref_idx)
        assert np.array_equal(sel.selected_scores.cpu().numpy(), ref_ss)


@pytest.mark.parametrize("strategy", ["least_confidence", "margin", "entropy"])
def test_uncertainty_steps_with_blocked_copy(cuda, strategy):
    """uncertainty_sampling.py:85-112 on one pool, three iterations: the first
    scores with the row-major kernel, the later ones build and read the blocked
    copy; every selection equals the oracle's for its shrinking unlabeled list."""
    from dal import uncertainty_sampling as us
    from dal.engine import PoolState
    from dal.forest import Forest

    n, d, k = 30_000, 256, 50
    X = O.synthetic_pool(n, d, seed=17)
    st = PoolState(X, device=cuda)
    F = Forest.synthetic(10, 4, d, seed=9)
    of = O.synthetic_forest(10, 4, d, seed=9)
    unl = np.arange(n)
    for it in range(3):
        sel = us.select(st, unl, F, k, strategy=strategy)
        _, ref_idx, ref_ss = O.uncertainty_select(X, unl, of, k, strategy)
        assert np.array_equal(sel.indices.cpu().numpy(), ref_idx), it
        assert np.array_equal(sel.selected_scores.cpu().numpy(), ref_ss), it
        assert (st._xb is not None) == (it > 0)
        unl = np.setdiff1d(unl, ref_idx)
