"""Fast level 1 of dal_dw_select (density_weighting.py:168,172 sortBy +
take): tau = the k-th smallest of the row groups' minimum pessimistic keys
bounds the k-th pessimistic key, and every row whose optimistic key is under
it becomes a candidate, instead of the 6-pass radix select + ordered
compaction.  The selection must be the oracle's, whether the bound keeps the
candidates under the capacity (the fast path stays enabled) or not (a forced
small capacity, or the top rows packed into a few groups: DAL_FLAG_SAMPLE_MISS,
exact re-run, the fast level 1 disabled for the pool), on one GPU and across
emulated shards; and the warm-step hipGraph must replay it exactly."""
import numpy as np
import pytest

from oracle import dal_oracle as O

pytestmark = pytest.mark.gpu


def _case(n, d, seed=0):
    X = O.synthetic_pool(n, d, seed=seed)
    of = O.synthetic_forest(10, 4, d, seed=1)
    E = np.arange(10)
    unl = np.arange(10, n)
    return X, of, E, unl


@pytest.mark.parametrize("n,d,k", [(100_000, 64, 100), (20_000, 32, 10), (5_000, 48, 100), (1_500, 16, 1),
                                   (250_000, 30, 1000), (100_000, 64, 1000)])
def test_fast_level1_select_bit_exact(cuda, n, d, k):
    from dal import density_weighting as dw
    from dal.engine import PoolState, level1_passes
    from dal.forest import Forest

    X, of, E, unl = _case(n, d)
    st = PoolState(X, excluded=E, device=cuda)
    assert level1_passes(st, n, k, 4096) > 0  # the fast level 1 is the path under test
    F = Forest.synthetic(10, 4, d, seed=1)
    ref_sc, ref_idx, ref_ss = O.density_select(X, unl, of, k, 1.0, E)
    for _ in range(2):  # cold, then warm
        sel = dw.select(st, unl, F, k)
        assert np.array_equal(sel.indices.cpu().numpy(), ref_idx)
        assert np.array_equal(sel.selected_scores.cpu().numpy(), ref_ss)
    assert st.level1_fast  # no overflow: every step took the fast level 1


def test_fast_level1_overflow_reruns_exactly(cuda):
    from dal import density_weighting as dw
    from dal.engine import PoolState
    from dal.forest import Forest

    X, of, E, unl = _case(50_000, 32, seed=5)
    st = PoolState(X, excluded=E, device=cuda)
    st.cap_base = 100  # capacity k: the group bound holds more candidates than that
    F = Forest.synthetic(10, 4, 32, seed=1)
    sel = dw.select(st, unl, F, 100)
    _, ref_idx, ref_ss = O.density_select(X, unl, of, 100, 1.0, E)
    assert np.array_equal(sel.indices.cpu().numpy(), ref_idx)
    assert np.array_equal(sel.selected_scores.cpu().numpy(), ref_ss)
    assert not st.level1_fast  # the overflow switched the pool to the exact level 1


def test_fast_level1_overflow_sharded(cuda):
    from dal import parallel
    from dal.forest import Forest

    n, d, world = 12_000, 24, 3
    X, of, E, unl = _case(n, d, seed=9)
    F = Forest.synthetic(10, 4, d, seed=1)
    sels = []
    for r in range(world):
        lo, hi, _ = parallel.shard_range(n, world, r)
        sels.append(parallel.ShardedSelector(X[lo:hi], n, r, world, excluded=E, device=cuda))
        sels[-1].state.cap_base = 50
    idx, sc = parallel.emulate(sels, unl, F, 50)
    _, ref_idx, ref_ss = O.density_select(X, unl, of, 50, 1.0, E)
    assert np.array_equal(idx.cpu().numpy(), ref_idx)
    assert np.array_equal(sc.cpu().numpy(), ref_ss)
    assert not all(s.state.level1_fast for s in sels)


def test_fast_level1_top_rows_in_few_groups(cuda):
    """The best rows packed at the front of the pool (a sorted pool): the k-th
    group minimum then lies far above the k-th key, the candidates overflow
    and the step re-runs exactly -- same selection as the oracle."""
    from dal import density_weighting as dw
    from dal.engine import PoolState
    from dal.forest import Forest

    n, d, k = 60_000, 32, 100
    X0, of, E, unl = _case(n, d, seed=23)
    ref_sc0, _, _ = O.density_select(X0, unl, of, k, 1.0, E)
    s_full = np.full(n, -np.inf)
    s_full[unl] = np.nan_to_num(ref_sc0, nan=-np.inf)
    order = np.argsort(-s_full, kind="stable")  # best rows first
    X = np.ascontiguousarray(X0[order])
    F = Forest.synthetic(10, 4, d, seed=1)
    _, ref_idx, ref_ss = O.density_select(X, unl, of, k, 1.0, E)
    st = PoolState(X, excluded=E, device=cuda)
    for _ in range(2):
        sel = dw.select(st, unl, F, k)
        assert np.array_equal(sel.indices.cpu().numpy(), ref_idx)
        assert np.array_equal(sel.selected_scores.cpu().numpy().view(np.int64), ref_ss.view(np.int64))


@pytest.mark.parametrize("n,d,k", [(30_000, 32, 10), (8_000, 64, 100)])
def test_warm_graph_al_iterations_bit_exact(cuda, n, d, k):
    """Warm steps replay a hipGraph: across AL iterations (a new forest and a
    shrinking unlabeled set each time) the selections equal the oracle's and
    the eager path's, and the per-row scores/votes are snapshots that the next
    replay does not overwrite."""
    from dal import engine
    from dal.forest import Forest

    X, _, E, unl = _case(n, d, seed=11)
    st = engine.PoolState(X, excluded=E, device=cuda)
    eager = engine.PoolState(X, excluded=E, device=cuda)
    eager.use_graphs = False
    prev = None
    for it in range(4):
        F = Forest.synthetic(10, 4, d, seed=100 + it)
        of = O.synthetic_forest(10, 4, d, seed=100 + it)
        sel = engine.density_step(st, unl, F, k)
        ref = engine.density_step(eager, unl, F, k)
        ref_sc, ref_idx, ref_ss = O.density_select(X, unl, of, k, 1.0, E)
        assert np.array_equal(sel.indices.cpu().numpy(), ref_idx)
        assert np.array_equal(sel.selected_scores.cpu().numpy(), ref_ss)
        assert np.array_equal(sel.votes.cpu().numpy(), ref.votes.cpu().numpy())
        assert np.array_equal(sel.scores.cpu().numpy().view(np.int64), ref.scores.cpu().numpy().view(np.int64))
        if it > 0:
            assert len(st._graphs) >= 1  # warm steps went through the graph
        if prev is not None:  # the previous step's outputs survived this replay
            assert np.array_equal(prev[0].indices.cpu().numpy(), prev[1])
        prev = (sel, ref_idx)
        unl = np.setdiff1d(unl, ref_idx)


def test_warm_graph_outputs_survive_later_steps(cuda):
    """Copy-on-write of the graph's per-row buffers: a Selection kept across
    later warm steps still reads its own votes and scores."""
    from dal import engine
    from dal.forest import Forest

    X, _, E, unl = _case(6_000, 16, seed=3)
    st = engine.PoolState(X, excluded=E, device=cuda)
    eager = engine.PoolState(X, excluded=E, device=cuda)
    eager.use_graphs = False
    engine.density_step(st, unl, Forest.synthetic(10, 4, 16, seed=7), 20)  # cold
    kept, refs = [], []
    for it in range(3):
        F = Forest.synthetic(10, 4, 16, seed=20 + it)
        kept.append(engine.density_step(st, unl, F, 20))  # nothing read yet
        refs.append(engine.density_step(eager, unl, F, 20))
    for a, b in zip(kept, refs):
        assert np.array_equal(a.votes.cpu().numpy(), b.votes.cpu().numpy())
        assert np.array_equal(a.scores.cpu().numpy().view(np.int64), b.scores.cpu().numpy().view(np.int64))
        assert np.array_equal(a.indices.cpu().numpy(), b.indices.cpu().numpy())


@pytest.mark.parametrize("n,d,trees,passes", [(100_000, 64, 10, 1), (284_807 // 4, 30, 100, 1),
                                              (100_000, 256, 10, 1), (20_000, 32, 10, 0),
                                              (3_000, 16, 7, 1), (300_000, 64, 10, 1)])
def test_dw_step_matches_separate_calls(cuda, n, d, trees, passes):
    """dal_dw_step (the score kernel writes the row-group minima -- one group
    per block, or several blocks folded by atomic max at 300,000 x 64 -- then
    ONE launch: tau, the append with the in-place re-rank, the last-block sort
    with the capacity check and the clears) gives the same bits as
    dal_forest_score + dal_dw_select, call after call on one workspace with
    DAL_STEP_WS_CLEAN (the folded minima must be left zero for the next call),
    and DAL_STEP_RESET_STATUS clears a stale status word."""
    import torch

    from dal import _lib, engine
    from dal._lib import DAL_STEP_RESET_STATUS, DAL_STEP_WS_CLEAN, call
    from dal.forest import Forest

    X = O.synthetic_pool(n, d, seed=4)
    E = np.arange(10)
    unl = np.arange(10, n)
    st = engine.PoolState(X, excluded=E, device=cuda)
    st.density_fixed()
    dens, colsum, norm64 = st.density_fixed(), st.colsum(), st.norms()
    flags, _, _ = st.row_flags(unl)
    k = 100
    cap = engine.candidate_cap(n, k)
    lib = _lib.load()
    lut = engine.device_lut("entropy", trees, cuda)
    derr = engine.density_error(st)
    P = lambda t: t.data_ptr()  # noqa: E731
    S = torch.cuda.current_stream(cuda).cuda_stream
    for it in range(3):
        F = Forest.synthetic(trees, 4, d, seed=40 + it)
        inner, leaf = F.device(cuda)
        # reference: the two calls
        v0, s0, klo0, khi0 = engine.forest_score(st, F, lut, flags, _lib.DAL_DESCENDING, density=dens,
                                                 density_err=derr, want_hi=True)
        wsb = int(lib.dal_dw_select_workspace_bytes(n, k, cap))
        ws0, wsp0 = engine.workspace(wsb, cuda)
        i0 = torch.empty(k, dtype=torch.int64, device=cuda)
        c0 = torch.empty(k, dtype=torch.float64, device=cuda)
        st.status.zero_()
        call("dal_dw_select", P(klo0), P(khi0), P(v0), P(flags), n, k, 0, P(lut), 1.0, P(st.x), d, d, P(norm64),
             P(colsum), cap, passes, wsp0, wsb, P(i0), P(c0), 0, P(st.status), 0, S)
        assert int(st.status.item()) == 0
        # the fused call, on one workspace zeroed once
        if it == 0:
            ws, wsp = engine.workspace(int(lib.dal_dw_step_workspace_bytes(n, k, cap)), cuda)
            ws.zero_()
        v = torch.empty(n, dtype=torch.int32, device=cuda)
        s = torch.empty(n, dtype=torch.float64, device=cuda)
        klo = torch.empty(n, dtype=torch.int64, device=cuda)
        khi = torch.empty(n, dtype=torch.int64, device=cuda)
        i1 = torch.empty(k, dtype=torch.int64, device=cuda)
        c1 = torch.empty(k, dtype=torch.float64, device=cuda)
        ok1 = torch.empty(k, dtype=torch.int64, device=cuda)
        st.status.fill_(_lib.DAL_FLAG_CAND_OVERFLOW)  # stale: the step must clear it on the device
        call("dal_dw_step", P(st.x), 0, 0, n, d, d, P(inner), P(leaf), trees, 4, P(lut), P(dens), float(derr), P(flags),
             1.0, 0, P(norm64), P(colsum), k, cap, passes, DAL_STEP_RESET_STATUS | DAL_STEP_WS_CLEAN, wsp,
             int(lib.dal_dw_step_workspace_bytes(n, k, cap)), P(v), P(s), P(klo), P(khi), P(i1), P(c1), P(ok1),
             P(st.status), 0, S)
        assert int(st.status.item()) == 0
        assert torch.equal(v, v0)
        assert torch.equal(s.view(torch.int64), s0.view(torch.int64))
        assert torch.equal(klo, klo0) and torch.equal(khi, khi0)
        assert torch.equal(i1, i0)
        assert torch.equal(c1.view(torch.int64), c0.view(torch.int64))
        hdr = ws[(wsp - ws.data_ptr()):(wsp - ws.data_ptr()) + 49312]  # sizeof(TopkHdr)
        assert int(hdr.count_nonzero()) == 0  # the header is left zero for the next call


def test_dw_step_sample_miss_flag(cuda):
    """A fast level 1 over capacity raises DAL_FLAG_SAMPLE_MISS from the
    last-block sort (the engine then re-runs with the exact level 1)."""
    import torch

    from dal import _lib, engine
    from dal._lib import call
    from dal.forest import Forest

    n, d, k = 50_000, 32, 100
    X = O.synthetic_pool(n, d, seed=5)
    st = engine.PoolState(X, excluded=np.arange(10), device=cuda)
    dens, colsum, norm64 = st.density_fixed(), st.colsum(), st.norms()
    flags, _, _ = st.row_flags(np.arange(10, n))
    F = Forest.synthetic(10, 4, d, seed=1)
    inner, leaf = F.device(cuda)
    lut = engine.device_lut("entropy", 10, cuda)
    lib = _lib.load()
    cap = k  # the group bound holds more candidates than k
    wsb = int(lib.dal_dw_step_workspace_bytes(n, k, cap))
    ws, wsp = engine.workspace(wsb, cuda)
    P = lambda t: t.data_ptr()  # noqa: E731
    outs = [torch.empty(n, dtype=t, device=cuda) for t in (torch.int32, torch.float64, torch.int64, torch.int64)]
    i1 = torch.empty(k, dtype=torch.int64, device=cuda)
    c1 = torch.empty(k, dtype=torch.float64, device=cuda)
    st.status.zero_()
    call("dal_dw_step", P(st.x), 0, 0, n, d, d, P(inner), P(leaf), 10, 4, P(lut), P(dens), float(engine.density_error(st)),
         P(flags), 1.0, 0, P(norm64), P(colsum), k, cap, 1, 0, wsp, wsb, *[P(t) for t in outs], P(i1), P(c1), 0,
         P(st.status), 0, torch.cuda.current_stream(cuda).cuda_stream)
    assert int(st.status.item()) & _lib.DAL_FLAG_SAMPLE_MISS


@pytest.mark.parametrize("n_distinct", [8, 300])
def test_many_candidates_and_ties(cuda, n_distinct):
    """Candidate lists above 1,024 take the block radix select before the
    one-block sort: with few distinct rows (massive exact ties: the k-th key's
    bucket never shrinks, full-sort fallback) and with many (the select
    path), cold and warm (plan) steps equal the oracle, ties to the lower index."""
    from dal import density_weighting as dw
    from dal.engine import PoolState
    from dal.forest import Forest

    n, d, k = 20_000, 32, 150
    base = O.synthetic_pool(n_distinct, d, seed=21)
    rng = np.random.default_rng(5)
    X = base[rng.integers(0, n_distinct, size=n)]
    of = O.synthetic_forest(10, 4, d, seed=1)
    F = Forest.synthetic(10, 4, d, seed=1)
    E = np.arange(10)
    unl = np.arange(10, n)
    _, ref_idx, ref_ss = O.density_select(X, unl, of, k, 1.0, E)
    st = PoolState(X, excluded=E, device=cuda)
    for _ in range(2):  # cold (dal_dw_step), then warm (dal_dw_plan)
        sel = dw.select(st, unl, F, k)
        assert np.array_equal(sel.indices.cpu().numpy(), ref_idx)
        assert np.array_equal(sel.selected_scores.cpu().numpy().view(np.int64), ref_ss.view(np.int64))


def test_warm_plan_exact_level1_and_capacity_growth(cuda):
    """Warm steps through dal_dw_plan when the fast level 1 overflows
    (the plan is rebuilt with the exact level 1: dal_dw_select inside the
    graph + the publishing kernel) and when the re-rank capacity must grow:
    every step equals the oracle, and the pool keeps the modes it fell back to."""
    from dal import engine
    from dal.forest import Forest

    X, _, E, unl = _case(40_000, 32, seed=13)
    st = engine.PoolState(X, excluded=E, device=cuda)
    st.cap_base = 100  # capacity k: the group bound overflows the fast level 1
    k = 100
    for it in range(3):
        F = Forest.synthetic(10, 4, 32, seed=200 + it)
        of = O.synthetic_forest(10, 4, 32, seed=200 + it)
        sel = engine.density_step(st, unl, F, k)
        _, ref_idx, ref_ss = O.density_select(X, unl, of, k, 1.0, E)
        assert np.array_equal(sel.indices.cpu().numpy(), ref_idx)
        assert np.array_equal(sel.selected_scores.cpu().numpy().view(np.int64), ref_ss.view(np.int64))
        unl = np.setdiff1d(unl, ref_idx)
    assert not st.level1_fast
    assert len(st._graphs) >= 1  # the warm steps went through a plan


@pytest.mark.gpu
def test_warm_plan_marking(cuda):
    """The plan's per-step marking: the marking kernel's arguments (list
    address, length, step stamp) are rewritten before every replay with
    hipGraphExecKernelNodeSetParams.  The unlabeled list shrinks every step
    (stale stamps of earlier steps must not count) and the selections equal
    the oracle's."""
    from dal import engine
    from dal.forest import Forest

    X, _, E, unl = _case(30_000, 64, seed=17)
    st = engine.PoolState(X, excluded=E, device=cuda)
    F = Forest.synthetic(10, 4, 64, seed=31)
    of = O.synthetic_forest(10, 4, 64, seed=31)
    k = 64
    for it in range(5):
        sel = engine.density_step(st, unl, F, k)
        _, ref_idx, ref_ss = O.density_select(X, unl, of, k, 1.0, E)
        assert np.array_equal(sel.indices.cpu().numpy(), ref_idx), it
        assert np.array_equal(sel.selected_scores.cpu().numpy().view(np.int64), ref_ss.view(np.int64)), it
        unl = np.setdiff1d(unl, ref_idx)[: max(k, len(unl) - 3000)]
    assert len(st._graphs) >= 1


class _OneShotComm:
    """all_gather of an already gathered [P, w] tensor (the merge alone)."""

    def __init__(self, g):
        self.g = g

    def all_gather(self, t):
        return self.g


@pytest.mark.gpu
@pytest.mark.parametrize("n_ranks,k,pad", [(1, 5, 0), (3, 100, 0), (8, 1000, 0), (4, 64, 40), (5, 7, 7)])
def test_topk_merge_packed(cuda, n_ranks, k, pad):
    """dal_topk_merge over a packed all-gather equals the (key, rank-major
    position) merge: per-rank lists sorted by (key, index), ranks in row
    order, many tied keys, padding keys at the tail, statuses OR-ed."""
    import torch

    from dal import _lib, parallel

    rng = np.random.default_rng(n_ranks * 1000 + k)
    none = np.uint64(_lib.DAL_KEY_NONE)
    rows = []
    keys_all, idx_all, sc_all = [], [], []
    for r in range(n_ranks):
        keys = np.sort(rng.integers(0, 50, size=k).astype(np.uint64) * np.uint64(1 << 40))
        idx = r * 100_000 + np.sort(rng.choice(100_000, size=k, replace=False)).astype(np.int64)
        if pad:
            keys[k - pad:] = none
            idx[k - pad:] = -1
        sc = rng.random(k)
        st = np.int64(1 << r if r < 3 else 0)
        rows.append(np.concatenate([keys.view(np.int64), idx, sc.view(np.int64), [st]]))
        keys_all.append(keys)
        idx_all.append(idx)
        sc_all.append(sc)
    g = torch.from_numpy(np.stack(rows)).to(cuda)
    K, I, S = np.concatenate(keys_all), np.concatenate(idx_all), np.concatenate(sc_all)
    order = np.lexsort((np.arange(K.size), K))[:k]
    valid = K[order] != none
    top = parallel.LocalTopk(g[0, :k], g[0, k:2 * k], g[0, 2 * k:3 * k].contiguous().view(torch.float64))
    status = g[0, 3 * k:3 * k + 1].to(torch.int32)
    for all_valid in ((True, False) if not pad else (False,)):
        (oi, os_), st = parallel.merge_packed(_OneShotComm(g), top, status, k, all_valid=all_valid)
        want = order if all_valid else order[valid]
        assert np.array_equal(oi.cpu().numpy(), I[want])
        assert np.array_equal(os_.cpu().numpy().view(np.int64), S[want].view(np.int64))
        assert st == sum(1 << r for r in range(min(n_ranks, 3)))


def _crafted_select(cuda, n, d, special, key_special, k, cap, seed=29):
    """dal_dw_select's fast level 1 on crafted interval keys: the rows in
    ``special`` carry the point key ``key_special``, every other row a larger
    one, so tau = key_special and exactly those rows are candidates.  Returns
    (selected indices, scores, status, expected indices, expected scores) --
    the expectation is the canonical fp64 top-k over the special rows."""
    import torch

    from dal import _lib, engine
    from dal._lib import call

    X = O.synthetic_pool(n, d, seed=seed)
    E = np.arange(10)
    st = engine.PoolState(X, excluded=E, device=cuda)
    colsum, norm64 = st.colsum(), st.norms()
    flags, _, _ = st.row_flags(np.arange(10, n))
    rng = np.random.default_rng(seed)
    votes_h = rng.integers(0, 11, size=n).astype(np.int32)
    lut_h = O.lut_entropy(10)
    keys_h = np.full(n, key_special + 1000, dtype=np.uint64)
    keys_h[special] = key_special
    keys = torch.from_numpy(keys_h.view(np.int64)).to(cuda)
    votes = torch.from_numpy(votes_h).to(cuda)
    lut = torch.from_numpy(lut_h).to(cuda)
    lib = _lib.load()
    wsb = int(lib.dal_dw_select_workspace_bytes(n, k, cap))
    ws, wsp = engine.workspace(wsb, cuda)
    ws.zero_()
    out_i = torch.empty(k, dtype=torch.int64, device=cuda)
    out_s = torch.empty(k, dtype=torch.float64, device=cuda)
    st.status.zero_()
    P = lambda t: t.data_ptr()  # noqa: E731
    call("dal_dw_select", P(keys), P(keys), P(votes), P(flags), n, k, 0, P(lut), 1.0, P(st.x), d, d, P(norm64),
         P(colsum), cap, 1, wsp, wsb, P(out_i), P(out_s), 0, P(st.status), 0,
         torch.cuda.current_stream(cuda).cuda_stream)
    status = int(st.status.item())
    dens = O.density_canonical(X, excluded=E)
    sc = lut_h[votes_h[special]] * dens[special]
    sc = np.where(np.isnan(sc), -np.inf, sc)
    order = np.lexsort((special, -sc))[:k]
    return out_i.cpu().numpy(), out_s.cpu().numpy(), status, np.asarray(special)[order], \
        (lut_h[votes_h] * dens)[np.asarray(special)[order]]


@pytest.mark.parametrize("layout,extra", [("per_group", 0), ("per_group", -1), ("one_region", 0),
                                          ("one_region", -1), ("local_sort_edge", 0)])
def test_fast_level1_region_and_capacity_boundaries(cuda, layout, extra):
    """The aperture-violation boundary shapes (DESIGN K3): 4,096 row groups
    of 64 rows, so summary_select_kernel runs its maximum of 128 blocks /
    candidate regions, with the candidate count exactly at ``cap`` (selection
    exact, no flag) and one past it (DAL_FLAG_SAMPLE_MISS, nothing read
    outside its region): one candidate in every group (every region 32), all
    candidates in one region (region count == cap), and regions of 256 / 257
    candidates (the local rank sort's limit)."""
    from dal import _lib

    n, d, gr = 4096 * 64, 16, 64
    if layout == "per_group":
        special = np.arange(4096) * gr + 17  # one per group: 128 regions x 32
        k = 100
    elif layout == "one_region":
        special = np.arange(10, 32 * gr)  # every row of block 0's 32 groups but E
        k = 10
    else:
        special = np.concatenate([np.arange(10, 10 + 256), 32 * gr + np.arange(257),
                                  np.arange(600, 4096) * gr + 5])  # block 0: 256, block 1: 257, then one per group
        k = 300
    cap = len(special) + extra
    if cap > _lib.DAL_SORT_CAP_PAYLOAD:
        pytest.skip("capacity above the fast level 1's one-block sort")
    idx, sc, status, ref_idx, ref_sc = _crafted_select(cuda, n, d, special, 1 << 40, k, cap)
    if extra < 0:
        assert status & _lib.DAL_FLAG_SAMPLE_MISS
        return
    assert status == 0
    assert np.array_equal(idx, ref_idx)
    assert np.array_equal(sc.view(np.int64), ref_sc.view(np.int64))


@pytest.mark.parametrize("n,d,trees", [(100_000, 64, 10), (300_000, 64, 10), (20_000, 32, 10)])
def test_dw_step_select_only_repeats_the_selection(cuda, n, d, trees):
    """DAL_STEP_KEEP_GROUPS leaves the folded row-group minima in the
    workspace and DAL_STEP_SELECT_ONLY re-runs only the selection launch on
    them (the bench times the fused step's selection this way): every repeat
    gives the full step's bits, and the last call without KEEP_GROUPS leaves
    the workspace as clean as a normal step (300,000 x 64: several score
    blocks per group, atomic-max minima; 20,000 x 32: the minima from the
    group_min pass)."""
    import torch

    from dal import _lib, engine
    from dal._lib import DAL_STEP_KEEP_GROUPS, DAL_STEP_SELECT_ONLY, DAL_STEP_WS_CLEAN, call
    from dal.forest import Forest

    X = O.synthetic_pool(n, d, seed=8)
    st = engine.PoolState(X, excluded=np.arange(10), device=cuda)
    dens, colsum, norm64 = st.density_fixed(), st.colsum(), st.norms()
    flags, _, _ = st.row_flags(np.arange(10, n))
    F = Forest.synthetic(trees, 4, d, seed=3)
    inner, leaf = F.device(cuda)
    lut = engine.device_lut("entropy", trees, cuda)
    lib = _lib.load()
    k = 100
    cap = engine.candidate_cap(n, k)
    wsb = int(lib.dal_dw_step_workspace_bytes(n, k, cap))
    ws, wsp = engine.workspace(wsb, cuda)
    ws.zero_()
    P = lambda t: t.data_ptr()  # noqa: E731
    bufs = [torch.empty(n, dtype=t, device=cuda) for t in (torch.int32, torch.float64, torch.int64, torch.int64)]
    S = torch.cuda.current_stream(cuda).cuda_stream

    def step(bits):
        i = torch.empty(k, dtype=torch.int64, device=cuda)
        c = torch.empty(k, dtype=torch.float64, device=cuda)
        st.status.zero_()
        call("dal_dw_step", P(st.x), 0, 0, n, d, d, P(inner), P(leaf), trees, 4, P(lut), P(dens),
             float(engine.density_error(st)), P(flags), 1.0, 0, P(norm64), P(colsum), k, cap, 1, bits, wsp, wsb,
             *[P(b) for b in bufs], P(i), P(c), 0, P(st.status), 0, S)
        assert int(st.status.item()) == 0
        return i, c

    i0, c0 = step(DAL_STEP_WS_CLEAN | DAL_STEP_KEEP_GROUPS)
    for _ in range(3):
        i1, c1 = step(DAL_STEP_WS_CLEAN | DAL_STEP_KEEP_GROUPS | DAL_STEP_SELECT_ONLY)
        assert torch.equal(i1, i0) and torch.equal(c1.view(torch.int64), c0.view(torch.int64))
    i1, c1 = step(DAL_STEP_WS_CLEAN | DAL_STEP_SELECT_ONLY)
    assert torch.equal(i1, i0)
    _, ref_idx, ref_ss = O.density_select(X, np.arange(10, n), O.synthetic_forest(trees, 4, d, seed=3), k, 1.0,
                                          np.arange(10))
    assert np.array_equal(i0.cpu().numpy(), ref_idx)
    # a normal step on the same workspace after the sequence: the minima were cleared
    i2, c2 = step(DAL_STEP_WS_CLEAN)
    assert torch.equal(i2, i0) and torch.equal(c2.view(torch.int64), c0.view(torch.int64))
    # flag combinations outside the contract are refused before any launch
    with pytest.raises(_lib.DalError):
        step(DAL_STEP_SELECT_ONLY)  # without WS_CLEAN
