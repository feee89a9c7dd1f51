"""GPU random-forest training (dal.random_forest, csrc/rf_train.hip) against
the CPU restatement of MLlib 2.1's RandomForest.trainClassifier
(oracle/rf_oracle.py; reference call sites final_thesis/uncertainty_sampling.py:71-76,
density_weighting.py:119-124).

Both sides take the same bootstrap weights and per-node feature subsets
(MLlib draws them from JVM RNGs); thresholds, split features, split
thresholds and leaf classes must then match bit for bit.  Parity unpinned at
the Spark boundary: no reference-held MLlib model exists (mllib/my_model/
holds only _SUCCESS markers)."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import dal_oracle as O
from oracle import rf_oracle as R

POS_INF_BITS = int(np.array([np.inf], dtype=np.float32).view(np.int32)[0])


# ------------------------------------------------------------ oracle (CPU) --
def test_oracle_find_splits_all_distinct_when_few():
    assert R.find_splits(np.array([3.0, 1.0, 2.0, 2.0, 1.0]), 31).tolist() == [1.0, 2.0, 3.0]


def test_oracle_find_splits_stride_rule():
    # 10 distinct values, numSplits 4: stride 2.0, thresholds where the running
    # count passes the running target (hand-evaluated)
    assert R.find_splits(np.arange(10.0), 4).tolist() == [1.0, 3.0, 5.0, 7.0]
    # duplicates: counts {0:5, 1:1, 2:1, 3:1, 4:2}, n = 10, numSplits 2 -> stride 10/3
    vals = np.array([0, 0, 0, 0, 0, 1, 2, 3, 4, 4], dtype=np.float64)
    assert R.find_splits(vals, 2).tolist() == [0.0, 2.0]


def test_oracle_num_splits_and_bins():
    assert R.num_splits(1000) == 31 and R.num_splits(2) == 1 and R.num_splits(1) == 0
    t = np.array([1.0, 3.0, 5.0])
    assert R.bin_values(np.array([0.5, 1.0, 2.0, 3.0, 6.0]), t).tolist() == [0, 0, 1, 1, 3]


def test_oracle_tree_separable_and_pure_children():
    X = np.array([[0.0], [1.0], [2.0], [3.0]])
    y = np.array([0, 0, 1, 1])
    thr, sf, st, lc = R.train_classifier(X, y, np.ones((1, 4), dtype=np.int64),
                                         np.zeros((1, 3, 1), dtype=np.int64), max_depth=2)
    assert sf[0].tolist() == [0, -1, -1] and st[0, 0] == 1.0
    assert lc[0].tolist() == [0, 0, 1, 1]  # pure children are leaves, classes padded


def test_oracle_tie_first_maximum_and_zero_gain_leaf():
    # both features separate perfectly: the first feature of the subset wins
    X = np.array([[0.0, 0.0], [1.0, 1.0]])
    y = np.array([0, 1])
    _, sf, _, _ = R.train_classifier(X, y, np.ones((1, 2), dtype=np.int64),
                                     np.array([[[1, 0]]]), max_depth=1)
    assert sf[0].tolist() == [1]
    # labels independent of x: every gain is 0 -> root leaf, class 0 on a tie
    X = np.array([[0.0], [0.0], [1.0], [1.0]])
    y = np.array([0, 1, 0, 1])
    _, sf, _, lc = R.train_classifier(X, y, np.ones((1, 4), dtype=np.int64),
                                      np.zeros((1, 1, 1), dtype=np.int64), max_depth=1)
    assert sf[0].tolist() == [-1] and lc[0].tolist() == [0, 0]


def test_bagging_inputs_shapes_and_determinism():
    from dal.random_forest import bagging_inputs, feature_subset_size

    w, s = bagging_inputs(100, 30, 10, 4, seed=3)
    w2, s2 = bagging_inputs(100, 30, 10, 4, seed=3)
    assert w.shape == (10, 100) and s.shape == (10, 15, 6)
    assert np.array_equal(w, w2) and np.array_equal(s, s2)
    assert all(len(set(row)) == 6 for row in s.reshape(-1, 6).tolist())
    w1, s1 = bagging_inputs(50, 7, 1, 3)
    assert (w1 == 1).all() and (s1 == np.arange(7)).all()
    assert feature_subset_size(784, 10) == 28 and feature_subset_size(30, 1) == 30


def test_split_histogram_limit_rejected_before_launch():
    """MLlib-valid inputs whose node histogram does not fit the
    split kernel's LDS are rejected with a clear error (Python) and with
    DAL_ERR_UNSUPPORTED before any HIP call (C ABI)."""
    import ctypes

    from dal import _lib
    from dal.random_forest import check_split_histogram

    check_split_histogram(600, 31)          # 600 x 33 x 8 = 158,400 B: fits
    check_split_histogram(80, 200)          # 80 x 202 x 8 = 129,280 B
    for m, ns in ((700, 31), (784, 31), (100, 254)):
        with pytest.raises(ValueError, match="split histogram"):
            check_split_histogram(m, ns)
    lib = _lib.load()
    p = ctypes.c_void_p(256)
    # numTrees=1 'auto' -> all 784 features at maxBins 32
    rc = lib.dal_rf_train(p, 1000, 784, 784, p, p, p, 31, p, p, 784, 1, 4, 1, 0.0, p, p, p, 1 << 30, None)
    assert rc == -3  # DAL_ERR_UNSUPPORTED


# ------------------------------------------------------------------- GPU --
def _oracle_heap(sf, st, lc):
    inner = np.zeros(sf.shape + (2,), dtype=np.int32)
    inner[..., 1] = POS_INF_BITS
    m = sf >= 0
    inner[..., 0][m] = sf[m]
    inner[..., 1][m] = st[m].astype(np.float32).view(np.int32)
    return inner, lc


def _datasets():
    out = []
    for name in ("checkerboard2x2.npz", "checkerboard4x4.npz", "rotated_checkerboard2x2.npz"):
        g = load_golden(name)
        out.append((name, g["X"], g["y"].astype(np.int64)))
    g = load_golden("unlabeled_init.npz")
    out.append(("unlabeled_init", g["X"], g["y"].astype(np.int64)))
    X = load_golden("synthetic_1500x30_T100.npz")["X"]
    out.append(("synthetic_1500x30", X, (X[:, 0] + 0.5 * X[:, 3] * X[:, 7] > 0.1).astype(np.int64)))
    X = load_golden("synthetic_512x64_T10.npz")["X"]
    out.append(("synthetic_512x64", X, (X[:, :8].sum(axis=1) > 4.0).astype(np.int64)))
    return out


DATASETS = _datasets()


@pytest.mark.gpu
@pytest.mark.parametrize("name,X,y", DATASETS, ids=[d[0] for d in DATASETS])
@pytest.mark.parametrize("trees,depth", [(10, 4), (1, 4), (100, 4), (7, 2), (5, 6)])
def test_gpu_train_matches_oracle(cuda, name, X, y, trees, depth):
    from dal.random_forest import bagging_inputs, train_classifier

    n, d = X.shape
    w, s = bagging_inputs(n, d, trees, depth, seed=trees + depth)
    F = train_classifier(X, y, trees, max_depth=depth, weights=w, feature_subsets=s, device=cuda)
    thr, sf, st, lc = R.train_classifier(X, y, w, s, max_depth=depth)
    inner, leaf = _oracle_heap(sf, st, lc)
    assert np.array_equal(F.inner, inner)
    assert np.array_equal(F.leaf, leaf)
    # the device thresholds per feature equal findSplitsForContinuousFeature
    t_dev, ns_dev = (a.cpu().numpy() for a in F.split_thresholds)
    for f in range(d):
        assert ns_dev[f] == thr[f].size
        assert np.array_equal(t_dev[f, :ns_dev[f]], thr[f].astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["uniform", "integers", "few", "normal16k", "tiny", "single"])
def test_gpu_find_splits_matches_oracle(cuda, case):
    import torch

    from dal import _lib
    from dal.random_forest import num_splits

    rng = np.random.default_rng(7)
    X = {"uniform": lambda: rng.random((5000, 3), dtype=np.float32),
         "integers": lambda: rng.integers(0, 10, (3000, 4)).astype(np.float32),
         "few": lambda: rng.integers(0, 3, (100, 2)).astype(np.float32),
         "normal16k": lambda: rng.standard_normal((16384, 2), dtype=np.float32),
         "tiny": lambda: np.array([[1.0, 5.0], [0.0, 5.0]], dtype=np.float32),
         "single": lambda: np.array([[2.0, -1.0]], dtype=np.float32)}[case]()
    n, d = X.shape
    ns = num_splits(n)
    x = torch.from_numpy(X).to(cuda)
    thr = torch.empty((d, _lib.DAL_RF_MAX_SPLITS), dtype=torch.float32, device=cuda)
    cnt = torch.empty(d, dtype=torch.int32, device=cuda)
    status = torch.zeros(1, dtype=torch.int32, device=cuda)
    _lib.call("dal_rf_find_splits", x.data_ptr(), n, d, d, 0, n, ns, thr.data_ptr(), cnt.data_ptr(),
              status.data_ptr(), torch.cuda.current_stream(cuda).cuda_stream)
    assert int(status.item()) == 0
    for f in range(d):
        ref = R.find_splits(X[:, f], ns)
        assert int(cnt[f]) == ref.size
        assert np.array_equal(thr[f, :ref.size].cpu().numpy(), ref.astype(np.float32))


@pytest.mark.gpu
def test_gpu_trained_forest_votes_and_predict(cuda):
    """The trained forest drives the selection kernels: votes equal the
    oracle's per-tree predict on the trained trees; predict = majority vote."""
    from dal.random_forest import bagging_inputs, predict, train_classifier

    g = load_golden("checkerboard4x4.npz")
    X, y = g["X"], g["y"].astype(np.int64)
    w, s = bagging_inputs(300, 2, 10, 4, seed=1)
    F = train_classifier(X[:300], y[:300], 10, weights=w, feature_subsets=s, device=cuda)
    _, sf, st, lc = R.train_classifier(X[:300], y[:300], w, s)
    of = R.heap_forest(sf, st, lc)
    labels, votes = predict(F, X, device=cuda)
    ref_votes = O.votes(of, X)
    assert np.array_equal(votes.cpu().numpy(), ref_votes)
    assert np.array_equal(labels.cpu().numpy(), (2 * ref_votes > 10).astype(np.uint8))
    assert (labels.cpu().numpy() == y).mean() > 0.5


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["min_instances", "min_gain", "bins4", "bins100", "depth1", "constant_feature",
                                  "one_class", "sampled_thresholds", "heavy_weights"])
def test_gpu_train_edge_cases_match_oracle(cuda, case):
    """MLlib's strategy knobs and degenerate inputs: minInstancesPerNode,
    minInfoGain, maxBins, depth 1, a constant feature, a single-class label
    set, thresholds fitted on a row sample (n > max(maxBins^2, 10000)), and
    large bootstrap counts."""
    from dal.random_forest import bagging_inputs, split_sample_rows, train_classifier

    rng = np.random.default_rng(17)
    n, d, T, depth = 3000, 12, 10, 4
    kw, okw, max_bins = {}, {}, 32
    X = rng.standard_normal((n, d)).astype(np.float32)
    y = (X[:, 0] + 0.3 * X[:, 1] > 0).astype(np.int64)
    if case == "min_instances":
        kw, okw = dict(min_instances_per_node=25), dict(min_instances=25)
    elif case == "min_gain":
        kw, okw = dict(min_info_gain=0.01), dict(min_info_gain=0.01)
    elif case == "bins4":
        max_bins = 4
    elif case == "bins100":
        max_bins = 100
    elif case == "depth1":
        depth = 1
    elif case == "constant_feature":
        X[:, 0] = 0.5
        X[:, 3] = -2.0
    elif case == "one_class":
        y = np.ones(n, dtype=np.int64)
    elif case == "sampled_thresholds":
        n = 20000
        X = rng.random((n, d), dtype=np.float32)
        y = (X[:, 2] > 0.4).astype(np.int64)
    w, s = bagging_inputs(n, d, T, depth, seed=5)
    if case == "heavy_weights":
        w = (w * 37).astype(np.int32)
    F = train_classifier(X, y, T, max_depth=depth, max_bins=max_bins, weights=w, feature_subsets=s,
                         device=cuda, seed=3, **kw)
    rows = split_sample_rows(n, max_bins, seed=3)
    if case == "sampled_thresholds":
        assert rows is not None and 0 < rows.size <= 16384
    _, sf, st, lc = R.train_classifier(X, y, w, s, max_depth=depth, max_bins=max_bins, split_rows=rows, **okw)
    inner, leaf = _oracle_heap(sf, st, lc)
    assert np.array_equal(F.inner, inner)
    assert np.array_equal(F.leaf, leaf)
