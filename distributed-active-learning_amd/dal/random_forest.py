"""GPU random-forest training: the drop-in for MLlib's
``RandomForest.trainClassifier`` on the AL loop's labeled set (SURVEY §8(f)
row 4).

Reference call sites (the per-iteration model fit):
  final_thesis/uncertainty_sampling.py:71-76
  final_thesis/density_weighting.py:119-124
      model = RandomForest.trainClassifier(train, numClasses=2,
                  categoricalFeaturesInfo={}, numTrees=T,
                  featureSubsetStrategy="auto", impurity='gini')   # maxDepth=4, maxBins=32

Every arithmetic step runs in libdal (csrc/rf_train.hip): threshold search
(findSplitsForContinuousFeature), binning, level-wise weighted Gini histograms
and split selection.  The host draws what MLlib draws from its JVM RNGs --
the Poisson(1) bootstrap weights and the per-node feature subsets -- with
numpy (seeded), so a fit is deterministic; the oracle (oracle/rf_oracle.py)
takes the same draws.  The result is a ``dal.forest.Forest`` in the heap
layout the selection kernels consume, already resident on the device.
"""
from __future__ import annotations

import math

import numpy as np

from . import _lib
from ._lib import (DAL_FLAG_RF_SPLITS, DAL_RF_MAX_DEPTH, DAL_RF_MAX_SPLIT_SAMPLE, DAL_RF_MAX_SPLITS,
                   DAL_RF_SPLIT_LDS_BYTES, call)
from .forest import Forest


def feature_subset_size(n_features: int, n_trees: int, strategy: str = "auto") -> int:
    """MLlib featureSubsetStrategy: "auto" = "all" for one tree, "sqrt" for a
    forest (classification); also "all", "sqrt", "log2", "onethird"."""
    if strategy == "auto":
        strategy = "all" if n_trees == 1 else "sqrt"
    if strategy == "all":
        return n_features
    if strategy == "sqrt":
        return int(math.ceil(math.sqrt(n_features)))
    if strategy == "log2":
        return max(1, int(math.ceil(math.log2(n_features))))
    if strategy == "onethird":
        return int(math.ceil(n_features / 3.0))
    raise ValueError(f"unknown featureSubsetStrategy {strategy!r}")


def bagging_inputs(n: int, d: int, n_trees: int, max_depth: int = 4, seed: int = 0,
                   feature_subset_strategy: str = "auto"):
    """(weights int32 [T, n], subsets int32 [T, 2^max_depth - 1, m]): Poisson(1)
    instance weights per tree (BaggedPoint with replacement when T > 1, all
    ones for a single tree) and the feature subset of every heap node (a
    random m-subset in draw order; all features in index order when m = d)."""
    rng = np.random.default_rng(seed)
    m = feature_subset_size(d, n_trees, feature_subset_strategy)
    if n_trees > 1:
        weights = rng.poisson(1.0, size=(n_trees, n)).astype(np.int32)
    else:
        weights = np.ones((1, n), dtype=np.int32)
    n_inner = (1 << max_depth) - 1
    if m == d:
        subsets = np.broadcast_to(np.arange(d, dtype=np.int32), (n_trees, n_inner, d)).copy()
    else:
        keys = rng.random((n_trees, n_inner, d))
        subsets = np.argsort(keys, axis=2, kind="stable")[:, :, :m].astype(np.int32)
    return weights, subsets


def split_sample_rows(n: int, max_bins: int = 32, seed: int = 0):
    """Rows the thresholds are fitted on.  MLlib uses every row when
    n <= max(maxBins^2, 10000), else a Bernoulli sample of expected size
    10000 (DecisionTree findSplits; its RNG differs, so parity is unpinned
    for that case).  None = all rows."""
    required = max(max_bins * max_bins, 10000)
    if n <= required and n <= DAL_RF_MAX_SPLIT_SAMPLE:
        return None
    rng = np.random.default_rng(seed + 0x5EED)
    rows = np.nonzero(rng.random(n) < min(required, DAL_RF_MAX_SPLIT_SAMPLE) / float(n))[0]
    return rows[:DAL_RF_MAX_SPLIT_SAMPLE].astype(np.int64)


def num_splits(n: int, max_bins: int = 32) -> int:
    """DecisionTreeMetadata: numBins = min(maxBins, numExamples), numSplits = numBins - 1."""
    return min(int(max_bins), int(n)) - 1


def _stream(device):
    import torch

    return torch.cuda.current_stream(device).cuda_stream


def check_split_histogram(m: int, n_splits: int) -> None:
    """dal_rf_train's split kernel holds one node's (feature slot, bin, class)
    histogram in LDS: m * (n_splits + 2) * 2 int32 counts must fit
    DAL_RF_SPLIT_LDS_BYTES.  MLlib itself has no such limit; raise a clear
    error instead of the kernel's DAL_ERR_UNSUPPORTED."""
    need = int(m) * (int(n_splits) + 2) * 8
    if need > DAL_RF_SPLIT_LDS_BYTES:
        raise ValueError(f"{m} candidate features per node x {n_splits + 1} thresholds need {need} bytes of "
                         f"split histogram, more than the GPU trainer's {DAL_RF_SPLIT_LDS_BYTES} "
                         "(lower max_bins or use a smaller feature subset)")


def train_classifier(X, y, num_trees: int = 10, max_depth: int = 4, max_bins: int = 32, seed: int = 0,
                     feature_subset_strategy: str = "auto", weights=None, feature_subsets=None,
                     min_instances_per_node: int = 1, min_info_gain: float = 0.0, device=None) -> Forest:
    """RandomForest.trainClassifier(numClasses=2, categoricalFeaturesInfo={},
    impurity='gini') on the GPU.  X [n, d] (numpy or torch), y labels in {0,1}.
    ``weights`` [T, n] / ``feature_subsets`` [T, 2^max_depth - 1, m] override
    the seeded draws (bagging_inputs)."""
    import torch

    from .engine import _require_cuda

    dev = _require_cuda(device)
    lib = _lib.load()
    x = X.to(device=dev, dtype=torch.float32) if isinstance(X, torch.Tensor) else \
        torch.from_numpy(np.ascontiguousarray(np.asarray(X, dtype=np.float32))).to(dev)
    x = x.contiguous()
    if x.dim() != 2 or x.shape[0] < 1:
        raise ValueError("training set must be a non-empty 2-D [rows, features] array")
    n, d = int(x.shape[0]), int(x.shape[1])
    if not 1 <= max_depth <= DAL_RF_MAX_DEPTH:
        raise ValueError(f"max_depth must lie in [1, {DAL_RF_MAX_DEPTH}]")
    if not 2 <= max_bins <= DAL_RF_MAX_SPLITS:
        raise ValueError(f"max_bins must lie in [2, {DAL_RF_MAX_SPLITS}]")
    yv = y.cpu().numpy() if isinstance(y, torch.Tensor) else np.asarray(y)
    yv = yv.reshape(-1)
    if yv.shape[0] != n or not np.isin(yv, (0, 1)).all():
        raise ValueError("labels must be n values in {0, 1}")
    labels = torch.from_numpy(yv.astype(np.uint8)).to(dev)
    if weights is None or feature_subsets is None:
        w_draw, s_draw = bagging_inputs(n, d, num_trees, max_depth, seed, feature_subset_strategy)
        weights = w_draw if weights is None else weights
        feature_subsets = s_draw if feature_subsets is None else feature_subsets
    w = torch.as_tensor(np.ascontiguousarray(weights, dtype=np.int32)).to(dev)
    sub = torch.as_tensor(np.ascontiguousarray(feature_subsets, dtype=np.int32)).to(dev)
    T = int(w.shape[0])
    n_inner = (1 << max_depth) - 1
    if tuple(w.shape) != (T, n) or sub.dim() != 3 or tuple(sub.shape[:2]) != (T, n_inner):
        raise ValueError(f"weights must be [T, {n}] and feature_subsets [T, {n_inner}, m]")
    m = int(sub.shape[2])
    if not 1 <= m <= d:
        raise ValueError("feature subsets must hold 1..d features")
    ns = num_splits(n, max_bins)
    check_split_histogram(m, ns)
    rows = split_sample_rows(n, max_bins, seed)
    n_sample = n if rows is None else int(rows.shape[0])
    rows_t = None if rows is None else torch.from_numpy(rows).to(dev)
    thresholds = torch.empty((d, DAL_RF_MAX_SPLITS), dtype=torch.float32, device=dev)
    n_splits = torch.empty(d, dtype=torch.int32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    s = _stream(dev)
    call("dal_rf_find_splits", x.data_ptr(), n, d, d, 0 if rows_t is None else rows_t.data_ptr(), n_sample, ns,
         thresholds.data_ptr(), n_splits.data_ptr(), status.data_ptr(), s)
    wsb = int(lib.dal_rf_train_workspace_bytes(n, d, T, max_depth, m, ns))
    ws = torch.empty(wsb + 256, dtype=torch.uint8, device=dev)
    wsp = (ws.data_ptr() + 255) // 256 * 256
    inner = torch.empty((T, n_inner, 2), dtype=torch.int32, device=dev)
    leaf = torch.empty((T, n_inner + 1), dtype=torch.uint8, device=dev)
    call("dal_rf_train", x.data_ptr(), n, d, d, labels.data_ptr(), thresholds.data_ptr(), n_splits.data_ptr(), ns,
         w.data_ptr(), sub.data_ptr(), m, T, max_depth, int(min_instances_per_node), float(min_info_gain),
         inner.data_ptr(), leaf.data_ptr(), wsp, wsb, s)
    if int(status.item()) & DAL_FLAG_RF_SPLITS:
        raise _lib.DalError("threshold search emitted more than num_splits + 1 thresholds")
    forest = Forest(inner=inner.cpu().numpy(), leaf=leaf.cpu().numpy(), depth=max_depth)
    forest._dev[str(dev)] = (inner, leaf)
    forest.split_thresholds = (thresholds, n_splits)
    return forest


def predict(forest: Forest, X, device=None):
    """RandomForestModel.predict (majority vote of the trees' hard labels;
    ties -> class 0) on the GPU: (labels uint8 [n], votes int32 [n])."""
    import torch

    from . import engine
    from ._lib import DAL_ASCENDING

    state = X if isinstance(X, engine.PoolState) else engine.PoolState(X, device=device)
    lut = engine.device_lut("least_confidence", forest.n_trees, state.device)
    votes, _, _, _ = engine.forest_score(state, forest, lut, state.flags, DAL_ASCENDING)
    return (2 * votes > forest.n_trees).to(torch.uint8), votes
