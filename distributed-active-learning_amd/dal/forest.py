"""Random-forest models in the device SoA layout used by ``dal_forest_score``.

Reference: the forest is ``RandomForest.trainClassifier(..., numTrees=T,
featureSubsetStrategy="auto", impurity='gini')`` (uncertainty_sampling.py:71-76,
density_weighting.py:119-124; MLlib default maxDepth=4) and the hot path walks
``model._java_model.trees()`` calling ``DecisionTreeModel(tree).predict``
(uncertainty_sampling.py:89-90).  MLlib 2.1 ``Node.predict`` sends a row left
when ``x[feature] <= threshold`` (continuous split) and a leaf returns its
class label.

Layout (per tree, complete binary heap of the forest's maximum depth D):
  inner[t][h] = (feature:int32, threshold:fp32 bits)   h < 2^D - 1
  leaf[t][l]  = class in {0,1}                          l < 2^D
Shallower leaves are padded with always-left splits (threshold = +inf) whose
whole subtree carries the leaf's class, so every root-to-leaf walk is exactly
D steps (wave-uniform trip count on the GPU).  Thresholds are rounded toward
-inf to fp32: for every fp32 x,  x <= t32  <=>  (double)x <= t64, so votes are
bit-exact against scikit-learn (fp32 X, fp64 thresholds) and against MLlib's
fp64 comparison FOR fp32-REPRESENTABLE FEATURE VALUES (the pool is fp32 here;
text features that are not fp32-representable are rounded on ingest, and a
value within that rounding of an fp64 MLlib threshold can fall on the other
side -- parity unpinned for such data: no reference-held model covers it).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from ._lib import DAL_MAX_TREE_DEPTH

_POS_INF_BITS = np.array([np.inf], dtype=np.float32).view(np.int32)[0]


def threshold_to_f32(t64: np.ndarray) -> np.ndarray:
    """Largest fp32 <= t64 (round toward -inf)."""
    t64 = np.asarray(t64, dtype=np.float64)
    with np.errstate(over="ignore"):
        f = t64.astype(np.float32)
    over = f.astype(np.float64) > t64
    f[over] = np.nextafter(f[over], np.float32(-np.inf))
    return f


@dataclass
class Forest:
    """A binary-classification forest of hard-voting trees (votes for class 1)."""

    inner: np.ndarray  # int32 [T, 2^D - 1, 2]
    leaf: np.ndarray  # uint8 [T, 2^D]
    depth: int
    _dev: dict = field(default_factory=dict, repr=False)

    @property
    def n_trees(self) -> int:
        return int(self.inner.shape[0])

    def check_features(self, d: int):
        """Raise unless every inner node tests a feature in [0, d): the score
        kernels index the pool row (or the blocked copy's feature list) with it."""
        if "range" not in self._dev:
            f = self.inner[..., 0]
            self._dev["range"] = (int(f.min()), int(f.max())) if f.size else (0, 0)
        lo, hi = self._dev["range"]
        if lo < 0 or hi >= d:
            raise ValueError(f"forest tests feature {lo if lo < 0 else hi}, outside the pool's {d} features")

    def device(self, device):
        """(inner, leaf) as device tensors, uploaded once per device."""
        import torch

        key = str(device)
        if key not in self._dev:
            self._dev[key] = (
                torch.from_numpy(np.ascontiguousarray(self.inner)).to(device),
                torch.from_numpy(np.ascontiguousarray(self.leaf)).to(device),
            )
        return self._dev[key]

    def blocked_prep(self, device, d: int):
        """The forest prepared for the blocked score kernel over d features
        (dal_forest_prepare, ABI v10: feature list, remapped nodes, leaves), a
        16-B aligned uint8 device tensor built once per (device, d) on the
        current stream -- or None when the blocked path does not apply."""
        import torch

        from . import _lib

        key = ("prep", str(device), int(d))
        if key not in self._dev:
            lib = _lib.load()
            nb = int(lib.dal_forest_prep_bytes(int(d), self.n_trees, self.depth))
            buf = None
            if nb:
                self.check_features(int(d))
                inner, leaf = self.device(device)
                buf = torch.empty(nb, dtype=torch.uint8, device=device)  # (caching allocator: 512-B aligned)
                _lib.call("dal_forest_prepare", inner.data_ptr(), leaf.data_ptr(), self.n_trees, self.depth,
                          int(d), buf.data_ptr(), nb,
                          torch.cuda.current_stream(device).cuda_stream)
            self._dev[key] = buf
        return self._dev[key]

    # ------------------------------------------------------------ builders
    @classmethod
    def from_nodes(cls, feature, threshold, left, right, value, roots) -> "Forest":
        """Flattened node arrays (global node ids): feature < 0 marks a leaf
        whose class is value[node]; internal nodes go to left[node] when
        x[feature] <= threshold[node] (fp64), else right[node]."""
        feature = np.asarray(feature, dtype=np.int64)
        threshold = np.asarray(threshold, dtype=np.float64)
        left = np.asarray(left, dtype=np.int64)
        right = np.asarray(right, dtype=np.int64)
        value = np.asarray(value, dtype=np.int64)
        roots = np.asarray(roots, dtype=np.int64)
        if roots.size == 0:
            raise ValueError("forest has no trees")

        def tree_depth(root):
            best, stack = 0, [(int(root), 0)]
            while stack:
                nd, lv = stack.pop()
                if feature[nd] < 0:
                    best = max(best, lv)
                else:
                    stack.append((int(left[nd]), lv + 1))
                    stack.append((int(right[nd]), lv + 1))
            return best

        D = max(1, max(tree_depth(r) for r in roots))
        if D > DAL_MAX_TREE_DEPTH:
            raise ValueError(f"tree depth {D} exceeds DAL_MAX_TREE_DEPTH={DAL_MAX_TREE_DEPTH}")
        n_inner, n_leaf = (1 << D) - 1, 1 << D
        T = roots.size
        inner = np.zeros((T, n_inner, 2), dtype=np.int32)
        inner[:, :, 1] = _POS_INF_BITS
        leaf = np.zeros((T, n_leaf), dtype=np.uint8)
        thr32 = threshold_to_f32(threshold).view(np.int32)
        for t, root in enumerate(roots):
            stack = [(int(root), 0, 0)]  # (node, heap index, level)
            while stack:
                nd, h, lv = stack.pop()
                if feature[nd] < 0:
                    cls_ = np.uint8(1 if value[nd] else 0)
                    # pad the subtree below heap position h with the leaf class
                    span = 1 << (D - lv)
                    first_leaf = (h + 1) * span - 1 - n_inner
                    leaf[t, first_leaf:first_leaf + span] = cls_
                    continue  # padded inner nodes keep (0, +inf): always left
                inner[t, h, 0] = feature[nd]
                inner[t, h, 1] = thr32[nd]
                stack.append((int(left[nd]), 2 * h + 1, lv + 1))
                stack.append((int(right[nd]), 2 * h + 2, lv + 1))
        return cls(inner=inner, leaf=leaf, depth=D)

    @classmethod
    def from_sklearn(cls, rf, positive_label=1) -> "Forest":
        """From a fitted ``sklearn.ensemble.RandomForestClassifier``: each tree
        votes 1 when its leaf's majority class equals ``positive_label``."""
        classes = np.asarray(rf.classes_)
        feat, thr, lft, rgt, val, roots = [], [], [], [], [], []
        base = 0
        for est in rf.estimators_:
            tr = est.tree_
            roots.append(base)
            cl = np.asarray(tr.children_left)
            cr = np.asarray(tr.children_right)
            is_leaf = cl < 0
            lab = classes[np.argmax(tr.value[:, 0, :], axis=1)]
            feat.append(np.where(is_leaf, -1, tr.feature))
            thr.append(np.where(is_leaf, 0.0, tr.threshold))
            lft.append(np.where(is_leaf, -1, cl + base))
            rgt.append(np.where(is_leaf, -1, cr + base))
            val.append(np.where(is_leaf, (lab == positive_label).astype(np.int64), 0))
            base += tr.node_count
        return cls.from_nodes(np.concatenate(feat), np.concatenate(thr), np.concatenate(lft),
                              np.concatenate(rgt), np.concatenate(val), np.array(roots))

    @classmethod
    def from_mllib_debug_string(cls, text: str) -> "Forest":
        """Parse MLlib's ``RandomForestModel.toDebugString()`` (Spark 2.1
        ``Node.subtreeToString``): ``Tree k:`` headers, ``If (feature f <= t)`` /
        ``Else (feature f > t)`` for continuous splits, ``Predict: c`` at leaves.
        Categorical splits are rejected (the reference uses
        ``categoricalFeaturesInfo={}``, uncertainty_sampling.py:73)."""
        import re

        lines = [ln.strip() for ln in text.splitlines() if ln.strip()]
        trees, cur = [], None
        for ln in lines:
            if re.match(r"^Tree \d+:$", ln):
                cur = []
                trees.append(cur)
            elif cur is not None and (ln.startswith("If ") or ln.startswith("Else ")
                                      or ln.startswith("Predict:")):
                cur.append(ln)
        if not trees:
            raise ValueError("no 'Tree k:' sections found in the debug string")
        feat, thr, lft, rgt, val, roots = [], [], [], [], [], []
        if_re = re.compile(r"^If \(feature (\d+) <= ([^)]+)\)$")
        else_re = re.compile(r"^Else \(feature (\d+) > ([^)]+)\)$")

        def new_node():
            feat.append(-1)
            thr.append(0.0)
            lft.append(-1)
            rgt.append(-1)
            val.append(0)
            return len(feat) - 1

        for body in trees:
            pos = 0

            def parse():
                nonlocal pos
                ln = body[pos]
                pos += 1
                nd = new_node()
                if ln.startswith("Predict:"):
                    val[nd] = 1 if float(ln.split(":", 1)[1]) == 1.0 else 0
                    return nd
                m = if_re.match(ln)
                if not m:
                    raise ValueError(f"unsupported split line {ln!r} (only continuous splits)")
                feat[nd], thr[nd] = int(m.group(1)), float(m.group(2))
                lft[nd] = parse()
                m2 = else_re.match(body[pos])
                if not m2 or int(m2.group(1)) != feat[nd]:
                    raise ValueError(f"malformed Else line {body[pos]!r}")
                pos += 1
                rgt[nd] = parse()
                return nd

            roots.append(parse())
        return cls.from_nodes(feat, thr, lft, rgt, val, roots)

    @classmethod
    def from_mllib_saved(cls, path: str) -> "Forest":
        """Read an MLlib ``RandomForestModel.save(sc, path)`` directory: Parquet
        ``NodeData`` rows (treeId, nodeId, predict{predict, prob}, impurity,
        isLeaf, split{feature, threshold, featureType, categories}, leftNodeId,
        rightNodeId, infoGain) under ``path/data``; continuous splits only."""
        import glob
        import os

        import pyarrow.parquet as pq

        data = os.path.join(path, "data") if os.path.isdir(os.path.join(path, "data")) else path
        files = sorted(glob.glob(os.path.join(data, "*.parquet")))
        if not files:
            raise ValueError(f"no parquet files under {data}")
        rows = []
        for f in files:
            rows.extend(pq.read_table(f).to_pylist())
        by_tree = {}
        for r in rows:
            by_tree.setdefault(int(r["treeId"]), {})[int(r["nodeId"])] = r
        feat, thr, lft, rgt, val, roots = [], [], [], [], [], []
        for t in sorted(by_tree):
            nodes = by_tree[t]
            gid = {nid: len(feat) + i for i, nid in enumerate(sorted(nodes))}
            for nid in sorted(nodes):
                r = nodes[nid]
                if r["isLeaf"]:
                    feat.append(-1)
                    thr.append(0.0)
                    lft.append(-1)
                    rgt.append(-1)
                    val.append(1 if float(r["predict"]["predict"]) == 1.0 else 0)
                else:
                    sp = r["split"]
                    if int(sp.get("featureType", 0)) != 0:
                        raise ValueError("categorical splits are not supported")
                    feat.append(int(sp["feature"]))
                    thr.append(float(sp["threshold"]))
                    lft.append(gid[int(r["leftNodeId"])])
                    rgt.append(gid[int(r["rightNodeId"])])
                    val.append(0)
            roots.append(gid[min(nodes)])  # MLlib root node id = 1 (smallest)
        return cls.from_nodes(feat, thr, lft, rgt, val, roots)

    @classmethod
    def synthetic(cls, n_trees: int, depth: int, n_features: int, seed: int = 1,
                  dist: str = "uniform") -> "Forest":
        """BASELINE.json synthetic forest: T complete depth-``depth`` trees,
        feature ~ U{0..D-1}, threshold ~ U(0,1) (or N(0,1)) as fp32, leaf
        class ~ Bernoulli(0.5) -- the same draw order as the test oracle."""
        rng = np.random.default_rng(seed)
        n_inner, n_leaf = (1 << depth) - 1, 1 << depth
        inner = np.zeros((n_trees, n_inner, 2), dtype=np.int32)
        leaf = np.zeros((n_trees, n_leaf), dtype=np.uint8)
        for t in range(n_trees):
            f = rng.integers(0, n_features, size=n_inner)
            if dist == "uniform":
                th = rng.random(n_inner).astype(np.float32)
            else:
                th = rng.standard_normal(n_inner).astype(np.float32)
            lv = rng.integers(0, 2, size=n_leaf)
            inner[t, :, 0] = f
            inner[t, :, 1] = th.view(np.int32)
            leaf[t] = lv
        return cls(inner=inner, leaf=leaf, depth=depth)
