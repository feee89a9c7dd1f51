"""Forest SoA conversion (dal.forest) -- host logic, CPU only.

The heap walk below is test infrastructure mirroring the kernel's traversal
(x <= thr -> 2h+1 else 2h+2) so the layout can be checked without a GPU.
"""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from conftest import golden_forest, load_golden
from dal.forest import Forest, threshold_to_f32
from oracle import dal_oracle as O


def heap_votes(F: Forest, X):
    X32 = np.asarray(X, dtype=np.float32)
    n = X32.shape[0]
    rows = np.arange(n)
    n_inner = (1 << F.depth) - 1
    v = np.zeros(n, dtype=np.int64)
    thr = F.inner[:, :, 1].view(np.float32)
    for t in range(F.n_trees):
        h = np.zeros(n, dtype=np.int64)
        for _ in range(F.depth):
            f = F.inner[t, h, 0]
            go_left = X32[rows, f] <= thr[t, h]
            h = 2 * h + np.where(go_left, 1, 2)
        v += F.leaf[t, h - n_inner]
    return v


@pytest.mark.parametrize("name,prefix", [("unlabeled_init.npz", "forest_"),
                                         ("checkerboard2x2.npz", "it1_forest_"),
                                         ("checkerboard2x2.npz", "it5_forest_"),
                                         ("checkerboard4x4.npz", "it5_forest_"),
                                         ("rotated_checkerboard2x2.npz", "it5_forest_"),
                                         ("synthetic_1500x30_T100.npz", "forest_")])
def test_heap_layout_votes_match_oracle(name, prefix):
    g = load_golden(name)
    of = golden_forest(g, prefix)
    F = Forest.from_nodes(of.feature, of.threshold, of.left, of.right, of.value, of.roots)
    assert F.depth <= 4 or prefix == "forest_"
    X = g["X"]
    assert np.array_equal(heap_votes(F, X), O.votes(of, X))


def test_from_sklearn_matches_oracle_export():
    from sklearn.ensemble import RandomForestClassifier

    rng = np.random.default_rng(0)
    X = rng.random((400, 6)).astype(np.float32)
    y = (X[:, 0] + X[:, 1] > 1).astype(int)
    rf = RandomForestClassifier(n_estimators=7, max_depth=6, random_state=3).fit(X, y)
    F = Forest.from_sklearn(rf)
    of = O.forest_from_sklearn(rf)
    assert np.array_equal(heap_votes(F, X), O.votes(of, X))
    hard = np.stack([e.predict(X) for e in rf.estimators_]).astype(int).sum(0)
    assert np.array_equal(heap_votes(F, X), hard)


def test_single_class_forest_votes():
    from sklearn.ensemble import RandomForestClassifier

    X = np.random.default_rng(1).random((20, 3)).astype(np.float32)
    rf = RandomForestClassifier(n_estimators=4, max_depth=4, random_state=0).fit(X, np.ones(20, int))
    F = Forest.from_sklearn(rf)
    assert F.depth == 1  # single leaves padded to one always-left split
    assert np.array_equal(heap_votes(F, X), np.full(20, 4))


@settings(max_examples=300, deadline=None)
@given(t=st.floats(allow_nan=False, width=64), x=st.floats(allow_nan=False, width=32))
def test_threshold_rounding_preserves_compare(t, x):
    t32 = threshold_to_f32(np.array([t]))[0]
    assert (np.float32(x) <= t32) == (float(np.float32(x)) <= t)


def test_depth_limit():
    # a chain of 17 splits
    n = 17
    feat = list(range(n)) + [-1] * (n + 1)
    left = [n + i for i in range(n)] + [-1] * (n + 1)
    right = [i + 1 for i in range(n - 1)] + [2 * n] + [-1] * (n + 1)
    with pytest.raises(ValueError):
        Forest.from_nodes([f if f >= 0 else -1 for f in feat], np.zeros(2 * n + 1), left, right,
                          np.zeros(2 * n + 1), [0])


def mllib_debug_string(of, kind="classifier"):
    """Render oracle node arrays in Spark 2.1's toDebugString format (test helper)."""
    out = [f"TreeEnsembleModel {kind} with {of.n_trees} trees", ""]

    def rec(nd, ind):
        pre = " " * ind
        if of.feature[nd] < 0:
            out.append(f"{pre}Predict: {float(of.value[nd])}")
            return
        f, t = int(of.feature[nd]), repr(float(of.threshold[nd]))
        out.append(f"{pre}If (feature {f} <= {t})")
        rec(of.left[nd], ind + 1)
        out.append(f"{pre}Else (feature {f} > {t})")
        rec(of.right[nd], ind + 1)

    for t, root in enumerate(of.roots):
        out.append(f"  Tree {t}:")
        rec(int(root), 4)
    return "\n".join(out) + "\n"


@pytest.mark.parametrize("name,prefix", [("checkerboard4x4.npz", "it5_forest_"),
                                         ("synthetic_1500x30_T100.npz", "forest_")])
def test_from_mllib_debug_string(name, prefix):
    g = load_golden(name)
    of = golden_forest(g, prefix)
    F = Forest.from_mllib_debug_string(mllib_debug_string(of))
    assert np.array_equal(heap_votes(F, g["X"]), O.votes(of, g["X"]))


def test_from_mllib_debug_string_rejects_categorical():
    txt = "  Tree 0:\n    If (feature 0 in {1.0,2.0})\n     Predict: 0.0\n" \
          "    Else (feature 0 not in {1.0,2.0})\n     Predict: 1.0\n"
    with pytest.raises(ValueError):
        Forest.from_mllib_debug_string(txt)


def write_mllib_saved(of, path):
    """Render oracle node arrays in MLlib RandomForestModel.save's layout
    (NodeData rows in two Parquet part files under path/data; node ids 1
    (root), 2i, 2i+1 as MLlib assigns them) -- test helper."""
    import pyarrow as pa
    import pyarrow.parquet as pq

    rows = []
    for t, root in enumerate(of.roots):
        def rec(nd, nid):
            leaf = of.feature[nd] < 0
            rows.append({
                "treeId": t, "nodeId": nid,
                "predict": {"predict": float(of.value[nd]) if leaf else 0.0, "prob": 1.0},
                "impurity": 0.0, "isLeaf": bool(leaf),
                "split": None if leaf else {"feature": int(of.feature[nd]),
                                            "threshold": float(of.threshold[nd]),
                                            "featureType": 0, "categories": []},
                "leftNodeId": None if leaf else 2 * nid,
                "rightNodeId": None if leaf else 2 * nid + 1,
                "infoGain": None if leaf else 0.1})
            if not leaf:
                rec(int(of.left[nd]), 2 * nid)
                rec(int(of.right[nd]), 2 * nid + 1)
        rec(int(root), 1)
    import os

    os.makedirs(os.path.join(path, "data"), exist_ok=True)
    half = len(rows) // 2
    pq.write_table(pa.Table.from_pylist(rows[:half]), os.path.join(path, "data", "part-0.parquet"))
    pq.write_table(pa.Table.from_pylist(rows[half:]), os.path.join(path, "data", "part-1.parquet"))


def test_from_mllib_saved_parquet(tmp_path):
    """MLlib RandomForestModel.save layout: NodeData rows in Parquet, node ids
    1 (root), 2i, 2i+1 as MLlib assigns them."""
    g = load_golden("synthetic_512x64_T10.npz")
    of = golden_forest(g)
    write_mllib_saved(of, str(tmp_path))
    F = Forest.from_mllib_saved(str(tmp_path))
    assert np.array_equal(heap_votes(F, g["X"]), O.votes(of, g["X"]))


def test_check_features_rejects_out_of_range():
    """Every score launch first checks that the forest's features index the
    pool's row (the kernels gather x[f] / the blocked copy's run of f)."""
    import numpy as np
    import pytest

    from dal.forest import Forest

    F = Forest.synthetic(3, 4, 20, seed=1)
    F.check_features(20)
    with pytest.raises(ValueError, match="outside"):
        F.check_features(int(F.inner[..., 0].max()))
    bad = F.inner.copy()
    bad[0, 0, 0] = -1
    with pytest.raises(ValueError, match="-1"):
        Forest(inner=bad, leaf=F.leaf.copy(), depth=F.depth).check_features(20)
    assert np.array_equal(F.inner, Forest.synthetic(3, 4, 20, seed=1).inner)
