"""Truncated level 1 of dal_dw_select (density_weighting.py:168,172 sortBy +
take): two radix digits bound the k-th pessimistic key and every row whose
optimistic key is under the bound becomes a candidate, instead of the 6-pass
radix select + ordered compaction.  The selection must be the oracle's,
whether the bound keeps the candidates under the capacity (the fast path
stays enabled) or not (a forced small capacity: DAL_FLAG_SAMPLE_MISS, exact
re-run, the fast level 1 disabled for the pool), on one GPU and across
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
                                   (250_000, 30, 1000)])
def test_truncated_level1_select_bit_exact(cuda, n, d, k):
    from dal import density_weighting as dw
    from dal.engine import PoolState, level1_passes
    from dal.forest import Forest

    X, of, E, unl = _case(n, d)
    st = PoolState(X, excluded=E, device=cuda)
    assert level1_passes(st, n, k, 4096) > 0  # the truncated level 1 is the path under test
    F = Forest.synthetic(10, 4, d, seed=1)
    ref_sc, ref_idx, ref_ss = O.density_select(X, unl, of, k, 1.0, E)
    for _ in range(2):  # cold, then warm
        sel = dw.select(st, unl, F, k)
        assert np.array_equal(sel.indices.cpu().numpy(), ref_idx)
        assert np.array_equal(sel.selected_scores.cpu().numpy(), ref_ss)
    assert st.level1_fast  # no overflow: every step took the truncated level 1


def test_truncated_level1_overflow_reruns_exactly(cuda):
    from dal import density_weighting as dw
    from dal.engine import PoolState
    from dal.forest import Forest

    X, of, E, unl = _case(50_000, 32, seed=5)
    st = PoolState(X, excluded=E, device=cuda)
    st.cap_base = 100  # capacity k: the bucket bound holds more candidates than that
    F = Forest.synthetic(10, 4, 32, seed=1)
    sel = dw.select(st, unl, F, 100)
    _, ref_idx, ref_ss = O.density_select(X, unl, of, 100, 1.0, E)
    assert np.array_equal(sel.indices.cpu().numpy(), ref_idx)
    assert np.array_equal(sel.selected_scores.cpu().numpy(), ref_ss)
    assert not st.level1_fast  # the overflow switched the pool to the exact level 1


def test_truncated_level1_overflow_sharded(cuda):
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
