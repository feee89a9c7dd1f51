"""CPU oracle for random-forest training -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` (and bench's cpu_baseline leg) may import this; the product
(``dal.random_forest``) never does and fails loudly without its HIP library.

Restates the per-iteration model fit of the reference,

    RandomForest.trainClassifier(train, numClasses=2, categoricalFeaturesInfo={},
                                 numTrees=T, featureSubsetStrategy="auto",
                                 impurity='gini', maxDepth=4, maxBins=32)
        final_thesis/uncertainty_sampling.py:71-76
        final_thesis/density_weighting.py:119-124

whose arithmetic lives in the un-vendored Apache Spark 2.1.0 MLlib jar
(derby.log:5; not in /root/reference, no JVM here).  Its published algorithm
(org.apache.spark.mllib.tree / ml.tree.impl.RandomForest, Spark 2.1) as
restated here, for continuous features and binary labels:

  splits   findSplitsForContinuousFeature: distinct sorted values with counts;
           if #distinct <= numSplits every distinct value is a threshold, else
           stride = n / (numSplits + 1) and a value becomes a threshold when
           adding the next value's count moves the running count further from
           the running target (target += stride after each threshold);
           numSplits = min(maxBins, numExamples) - 1
  bins     TreePoint.findBin: Arrays.binarySearch -> bin = #{thresholds < x};
           split k sends bin <= k (x <= threshold_k) left
  bagging  Poisson(1) instance weights per (tree, row) when numTrees > 1
           (BaggedPoint, subsamplingRate 1); all ones for one tree
  features "auto" -> "sqrt" for numTrees > 1: ceil(sqrt(D)) features per node
           (reservoir sample; the order is the evaluation order); "all" for 1 tree
  impurity Gini.calculate: impurity = 1; for each class: f = c/total;
           impurity -= f*f (0 when total == 0); count = (long) sum(stats)
  gain     calculateImpurityStats: invalid (gain = -Double.MaxValue) when a
           child's count < minInstancesPerNode (1); gain = impurity
           - (lc/tc)*imp_l - (rc/tc)*imp_r; invalid when gain < minInfoGain (0)
  best     maxBy(gain) over a feature's splits in index order, then over the
           node's features in subset order (first maximum wins)
  growth   level by level; a node is a leaf when gain <= 0 or it sits at
           maxDepth; a child is created as a leaf when it reaches maxDepth or
           its impurity is 0.0; predict = first index of the largest class
           count (class 0 on ties)

MLlib draws the bootstrap weights and the per-node feature subsets from its
own JVM RNGs (commons-math Poisson, XORShiftRandom), which cannot be
reproduced here: they are INPUTS of this oracle and of the GPU trainer, so the
two are compared on identical draws.  For numExamples > max(maxBins^2, 10000)
MLlib fits the thresholds on a Bernoulli row sample; the caller passes the
sample rows (parity unpinned for that case: the sample RNG differs).
Parity unpinned at the Spark boundary (no reference-held model to compare).
"""
from __future__ import annotations

import math

import numpy as np

INVALID_GAIN = -np.finfo(np.float64).max  # ImpurityStats.getInvalidImpurityStats: Double.MinValue


def num_splits(n_examples: int, max_bins: int = 32) -> int:
    """DecisionTreeMetadata: numBins = min(maxBins, numExamples); numSplits = numBins - 1."""
    return min(max_bins, int(n_examples)) - 1


def find_splits(values: np.ndarray, n_splits: int) -> np.ndarray:
    """findSplitsForContinuousFeature (Spark 2.1) over the sample of one feature."""
    values = np.asarray(values, dtype=np.float64)
    if values.size == 0:
        return np.zeros(0, dtype=np.float64)
    uniq, counts = np.unique(values, return_counts=True)
    if uniq.size <= n_splits:
        return uniq.copy()
    stride = float(values.size) / (n_splits + 1)
    out = []
    current = int(counts[0])
    target = stride
    for index in range(1, uniq.size):
        previous = current
        current += int(counts[index])
        previous_gap = abs(previous - target)
        current_gap = abs(current - target)
        if previous_gap < current_gap:
            out.append(uniq[index - 1])
            target += stride
    return np.asarray(out, dtype=np.float64)


def bin_values(x: np.ndarray, thresholds: np.ndarray) -> np.ndarray:
    """TreePoint.findBin: index of an equal threshold, else the insertion point."""
    return np.searchsorted(np.asarray(thresholds, dtype=np.float64), np.asarray(x, dtype=np.float64),
                           side="left")


def gini(counts) -> float:
    total = float(counts[0]) + float(counts[1])
    if total == 0:
        return 0.0
    imp = 1.0
    for c in counts:
        f = float(c) / total
        imp -= f * f
    return imp


def impurity_stats(left, right, parent_impurity: float, min_instances: int = 1,
                   min_info_gain: float = 0.0):
    """calculateImpurityStats -> (gain, left impurity, right impurity)."""
    lc = int(left[0] + left[1])
    rc = int(right[0] + right[1])
    if lc < min_instances or rc < min_instances:
        return INVALID_GAIN, None, None
    tc = lc + rc
    li, ri = gini(left), gini(right)
    lw = lc / float(tc)
    rw = rc / float(tc)
    gain = parent_impurity - lw * li - rw * ri
    if gain < min_info_gain:
        return INVALID_GAIN, None, None
    return gain, li, ri


def predict(counts) -> int:
    """indexOfLargestArrayElement (strict >: first maximum)."""
    return 0 if counts[1] <= counts[0] else 1


def train_tree(bins: np.ndarray, labels: np.ndarray, weights: np.ndarray, subsets: np.ndarray,
               n_splits_f: np.ndarray, max_depth: int, min_instances: int = 1,
               min_info_gain: float = 0.0):
    """One tree.  bins [n, d] (bin per feature), labels {0,1} [n], weights int
    [n], subsets [2^maxDepth - 1, m] feature ids per heap node (evaluation
    order), n_splits_f [d].  Returns heap arrays (split_feature [n_inner] (-1 =
    leaf/absent), split_bin [n_inner], leaf_class [n_leaf]) in the padded
    layout of dal.forest.Forest (a shallow leaf's class fills its subtree)."""
    n_inner = (1 << max_depth) - 1
    n_leaf = 1 << max_depth
    split_feature = np.full(n_inner, -1, dtype=np.int64)
    split_bin = np.zeros(n_inner, dtype=np.int64)
    leaf_class = np.zeros(n_leaf, dtype=np.uint8)
    labels = np.asarray(labels, dtype=np.int64)
    weights = np.asarray(weights, dtype=np.int64)
    node = np.zeros(bins.shape[0], dtype=np.int64)  # heap index of each row's node
    # open nodes at the current level: heap index -> preset leaf flag
    level_nodes = {0: False}
    for level in range(max_depth + 1):
        nxt = {}
        for h, preset_leaf in sorted(level_nodes.items()):
            rows = np.nonzero((node == h) & (weights > 0))[0]
            cnt = np.array([weights[rows][labels[rows] == 0].sum(), weights[rows][labels[rows] == 1].sum()],
                           dtype=np.int64)
            best_gain, best = INVALID_GAIN, None
            if not preset_leaf and level < max_depth:
                parent_imp = gini(cnt)
                for f in subsets[h]:
                    f = int(f)
                    ns = int(n_splits_f[f])
                    hist = np.zeros((ns + 1, 2), dtype=np.int64)
                    np.add.at(hist, (bins[rows, f], labels[rows]), weights[rows])
                    cum = np.cumsum(hist, axis=0)
                    for k in range(ns):
                        left = cum[k]
                        right = cnt - left
                        gain, li, ri = impurity_stats(left, right, parent_imp, min_instances, min_info_gain)
                        if gain > best_gain:
                            best_gain, best = gain, (f, k, li, ri)
            if preset_leaf or level == max_depth or best_gain <= 0:
                # leaf: its class fills the heap subtree below h
                span = 1 << (max_depth - level)
                first = (h + 1) * span - 1 - n_inner
                leaf_class[first:first + span] = predict(cnt)
                continue
            f, k, li, ri = best
            split_feature[h] = f
            split_bin[h] = k
            child_leaf = level + 1 == max_depth
            nxt[2 * h + 1] = child_leaf or li == 0.0
            nxt[2 * h + 2] = child_leaf or ri == 0.0
            go_right = bins[:, f] > k
            here = node == h
            node[here & ~go_right] = 2 * h + 1
            node[here & go_right] = 2 * h + 2
        level_nodes = nxt
        if not level_nodes:
            break
    return split_feature, split_bin, leaf_class


def feature_subset_size(n_features: int, n_trees: int) -> int:
    """featureSubsetStrategy "auto": sqrt for a forest, all for a single tree."""
    return n_features if n_trees == 1 else int(math.ceil(math.sqrt(n_features)))


def train_classifier(X: np.ndarray, y: np.ndarray, weights: np.ndarray, subsets: np.ndarray,
                     max_depth: int = 4, max_bins: int = 32, split_rows=None, min_instances: int = 1,
                     min_info_gain: float = 0.0):
    """RandomForest.trainClassifier on given bagging weights [T, n] and
    feature subsets [T, 2^maxDepth - 1, m].  Returns (thresholds per feature
    (list of fp64 arrays), split_feature [T, n_inner], split_threshold fp64
    [T, n_inner] (NaN where no split), leaf_class [T, n_leaf])."""
    X = np.asarray(X, dtype=np.float64)
    n, d = X.shape
    ns = num_splits(n, max_bins)
    sample = X if split_rows is None else X[np.asarray(split_rows)]
    thresholds = [find_splits(sample[:, f], ns) for f in range(d)]
    n_splits_f = np.array([t.size for t in thresholds], dtype=np.int64)
    bins = np.stack([bin_values(X[:, f], thresholds[f]) for f in range(d)], axis=1) if d else \
        np.zeros((n, 0), dtype=np.int64)
    T = weights.shape[0]
    n_inner = (1 << max_depth) - 1
    sf = np.full((T, n_inner), -1, dtype=np.int64)
    st = np.full((T, n_inner), np.nan)
    lc = np.zeros((T, 1 << max_depth), dtype=np.uint8)
    for t in range(T):
        f_, b_, l_ = train_tree(bins, y, weights[t], subsets[t], n_splits_f, max_depth, min_instances,
                                min_info_gain)
        sf[t], lc[t] = f_, l_
        for h in np.nonzero(f_ >= 0)[0]:
            st[t, h] = thresholds[f_[h]][b_[h]]
    return thresholds, sf, st, lc


def heap_forest(split_feature, split_threshold, leaf_class):
    """The trained heap arrays as an OracleForest (flat nodes) for the vote
    oracle: absent / leaf positions below a leaf become always-left splits
    (feature 0, threshold +inf), the padded layout of dal.forest.Forest."""
    from .dal_oracle import OracleForest

    T, n_inner = split_feature.shape
    feat, thr, left, right, val, roots = [], [], [], [], [], []
    for t in range(T):
        base = len(feat)
        roots.append(base)
        for h in range(n_inner):
            has = split_feature[t, h] >= 0
            feat.append(int(split_feature[t, h]) if has else 0)
            thr.append(float(split_threshold[t, h]) if has else np.inf)
            left.append(base + 2 * h + 1)
            right.append(base + 2 * h + 2)
            val.append(0)
        for c in leaf_class[t]:
            feat.append(-1)
            thr.append(0.0)
            left.append(-1)
            right.append(-1)
            val.append(int(c))
    return OracleForest(np.array(feat), np.array(thr), np.array(left), np.array(right), np.array(val),
                        np.array(roots))
