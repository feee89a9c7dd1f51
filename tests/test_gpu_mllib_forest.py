"""An MLlib-format forest drives the GPU path (VERDICT r2
item 8).  Forests are trained on the GPU (dal.random_forest, MLlib 2.1's
RandomForest.trainClassifier algorithm) on the reference's checkerboard
sets, rendered in MLlib 2.1's ``toDebugString`` text and ``NodeData`` Parquet
layout (early leaves as MLlib leaves, fp64 thresholds), re-imported with
Forest.from_mllib_debug_string / from_mllib_saved, and the re-imported
forests' GPU votes and uncertainty / density-weighted selections are checked
against the oracle on the same trees.

Reference: uncertainty_sampling.py:89 (``model._java_model.trees()``),
:88-109 (votes, LC score, sortBy, take), mllib/save_regression_model.py:28-33
(RandomForestModel.save / load), density_weighting.py:133-176.
No Spark-written model exists in the reference (mllib/my_model/ holds only
markers), so the renderings are the test's own: parity with Spark's writer is
unpinned beyond the documented formats.
"""
import numpy as np
import pytest

from conftest import load_golden
from oracle import dal_oracle as O
from test_forest_format import mllib_debug_string, write_mllib_saved

pytestmark = pytest.mark.gpu

E = np.arange(10)


def _np(t):
    return t.detach().cpu().numpy()


def heap_to_nodes(F):
    """GPU-trained heap forest -> MLlib-shaped node arrays: an inner node
    with threshold +inf (the trainer's early leaf: every row goes left) is
    collapsed into its left descendant, so early leaves are leaves as in
    MLlib's Node tree."""
    feat, thr, left, right, val, roots = [], [], [], [], [], []
    n_inner = (1 << F.depth) - 1
    thr32 = F.inner[:, :, 1].view(np.float32)

    def rec(t, h):
        nd = len(feat)
        feat.append(-1)
        thr.append(0.0)
        left.append(-1)
        right.append(-1)
        val.append(0)
        while h < n_inner and np.isposinf(thr32[t, h]):
            h = 2 * h + 1
        if h >= n_inner:
            val[nd] = int(F.leaf[t, h - n_inner])
            return nd
        feat[nd] = int(F.inner[t, h, 0])
        thr[nd] = float(thr32[t, h])
        left[nd] = rec(t, 2 * h + 1)
        right[nd] = rec(t, 2 * h + 2)
        return nd

    for t in range(F.n_trees):
        roots.append(rec(t, 0))
    return O.OracleForest(np.array(feat, np.int32), np.array(thr), np.array(left, np.int32),
                          np.array(right, np.int32), np.array(val, np.int32), np.array(roots, np.int32))


@pytest.mark.parametrize("name", ["checkerboard2x2.npz", "checkerboard4x4.npz", "rotated_checkerboard2x2.npz"])
@pytest.mark.parametrize("trees", [10, 100])
def test_mllib_format_forest_drives_gpu_selection(cuda, tmp_path, name, trees):
    from dal import density_weighting as dw
    from dal import uncertainty_sampling as us
    from dal.forest import Forest
    from dal.random_forest import predict, train_classifier

    g = load_golden(name)
    X, y = g["X"], g["y"].astype(np.int64)
    lab = np.arange(200)
    F_gpu = train_classifier(X[lab], y[lab], trees, max_depth=4, seed=3, device=cuda)
    of = heap_to_nodes(F_gpu)
    assert (of.feature < 0).any()  # MLlib-style leaves present
    F_txt = Forest.from_mllib_debug_string(mllib_debug_string(of))
    write_mllib_saved(of, str(tmp_path))
    F_pq = Forest.from_mllib_saved(str(tmp_path))
    ref_votes = O.votes(of, X)
    _, v_gpu = predict(F_gpu, X, device=cuda)
    assert np.array_equal(_np(v_gpu), ref_votes)
    unl = np.arange(200, X.shape[0])
    for F in (F_txt, F_pq):
        labels, votes = predict(F, X, device=cuda)
        assert np.array_equal(_np(votes), ref_votes)
        assert np.array_equal(_np(labels), (2 * ref_votes > trees).astype(np.uint8))
        for strategy in ("least_confidence", "entropy"):
            sel = us.select(X, unl, F, 10, strategy=strategy, device=cuda)
            _, o_idx, o_sc = O.uncertainty_select(X, unl, of, 10, strategy)
            assert np.array_equal(_np(sel.indices), o_idx)
            assert np.array_equal(_np(sel.selected_scores), o_sc, equal_nan=True)
        sel = dw.select(X, unl, F, 10, excluded_idx=E, device=cuda)
        _, o_idx, o_sc = O.density_select(X, unl, of, 10, 1.0, E)
        assert np.array_equal(_np(sel.indices), o_idx)
        assert np.array_equal(_np(sel.selected_scores), o_sc)
