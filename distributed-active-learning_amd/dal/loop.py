"""Active-learning loop driver and pool ingest.

Reproduces the end-to-end behaviour of the reference scripts around the
GPU query step:

  ingest     uncertainty_sampling.py:37-42 / density_weighting.py:45-53,59-65:
             whitespace text, label in the last column, -1 -> 0, optional
             take(n_samples) truncation
  loop       uncertainty_sampling.py:59-114, density_weighting.py:106-179,
             random_sampling.py:60-94: labeled = range(window_size) at start;
             each iteration trains a forest on the labeled rows, measures test
             accuracy, selects window_size rows and moves them to the labeled set;
             stops when the unlabeled set is empty
  log        ``labeled =  L  unlabeled =  U`` (:65) and
             ``Iteration  i  -- accu =  a`` (:113)

Forest training (RandomForest.trainClassifier, uncertainty_sampling.py:71-76)
runs on the GPU by default (dal.random_forest: MLlib 2.1's gini / maxDepth 4 /
maxBins 32 / sqrt-feature algorithm, seeded bagging draws); trainer="sklearn"
keeps the scikit-learn fit of round 1.  The selection step is the GPU path
(dal.uncertainty_sampling / dal.density_weighting).  The random baseline
(random_sampling.py:88-89, ``sortBy(np.random.uniform).take``) has no
arithmetic and runs on the host.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


def load_labeled_text(path: str, n_samples=None, label_map: str = "reference"):
    """Whitespace-separated rows, features then label.  label_map="reference"
    applies the scripts' ``0 if int(label) == -1 else 1`` (uncertainty_sampling.py:39,
    written for the +-1 striatum labels); "as_is" keeps 0/1 labels (the LAL
    checkerboard files).  Returns (X fp32 [N, D], y int64 [N]).  Parsed by the
    native multi-threaded parser (dal.ingest; dal.ingest.load_pool uploads the
    pool to HBM through pinned memory instead)."""
    from .ingest import parse_labeled_text

    return parse_labeled_text(path, n_samples=n_samples, label_map=label_map)


class GpuForestModel:
    """A forest trained by dal.random_forest, with MLlib's RandomForestModel
    ``predict`` (majority vote) on the GPU."""

    def __init__(self, forest, device=None):
        self.forest = forest
        self.device = device

    def predict(self, X):
        from .random_forest import predict

        labels, _ = predict(self.forest, X, device=self.device)
        return labels.cpu().numpy()


def train_forest(X, y, n_estimators: int = 10, seed: int = 0, max_depth: int = 4, trainer="gpu",
                 device=None):
    """RandomForest.trainClassifier(numTrees=T, featureSubsetStrategy='auto',
    impurity='gini') with MLlib's default maxDepth=4.  trainer: "gpu"
    (dal.random_forest), "sklearn", or a callable (X, y, T, seed) -> model with
    ``predict``."""
    if callable(trainer):
        return trainer(X, y, n_estimators, seed)
    if trainer == "gpu":
        from .random_forest import train_classifier

        return GpuForestModel(train_classifier(X, y, n_estimators, max_depth=max_depth, seed=seed,
                                               device=device), device)
    if trainer != "sklearn":
        raise ValueError(f"unknown trainer {trainer!r}")
    from sklearn.ensemble import RandomForestClassifier

    rf = RandomForestClassifier(n_estimators=n_estimators, max_depth=max_depth,
                                max_features="sqrt", bootstrap=True, random_state=seed)
    rf.fit(X, y)
    return rf


@dataclass
class LoopResult:
    labeled_history: list = field(default_factory=list)  # selected indices per iteration
    accuracy: list = field(default_factory=list)  # test accuracy (%) per iteration
    log: list = field(default_factory=list)


def run_loop(X, y, X_test=None, y_test=None, strategy: str = "uncertainty",
             window_size: int = 10, n_estimators: int = 10, max_iterations=None,
             seed: int = 0, select_fn=None, device=None, beta: float = 1.0,
             verbose: bool = False, trainer="gpu") -> LoopResult:
    """Run the AL loop.  strategy: "uncertainty" (uncertainty_sampling.py),
    "density" (density_weighting.py, E = L0 = range(window_size)) or "random".
    trainer: see train_forest.

    ``select_fn(strategy, pool, unlabeled, model, k) -> indices`` can replace
    the GPU step (tests use the oracle); by default the dal GPU path runs.
    """
    from .forest import Forest

    n = X.shape[0]
    labeled = list(range(min(window_size, n)))
    unlabeled = np.arange(len(labeled), n, dtype=np.int64)
    res = LoopResult()
    rng = np.random.default_rng(seed)
    state = test_state = None
    if select_fn is None and strategy != "random":
        from .engine import PoolState

        excluded = np.arange(len(labeled)) if strategy == "density" else None
        state = PoolState(X, excluded=excluded, device=device)
    it = 1
    while True:
        line = f"labeled =  {len(labeled)}  unlabeled =  {unlabeled.size}"
        res.log.append(line)
        if verbose:
            print(line)
        if unlabeled.size == 0:
            break
        if max_iterations is not None and it > max_iterations:
            break
        lab = np.asarray(labeled)
        rf = train_forest(X[lab], y[lab], n_estimators, seed + it, trainer=trainer, device=device)
        acc = None
        if X_test is not None:
            if isinstance(rf, GpuForestModel) and test_state is None:
                from .engine import PoolState

                test_state = PoolState(X_test, device=device)  # uploaded once
            pred = rf.predict(test_state if isinstance(rf, GpuForestModel) else X_test)
            acc = (1 - np.mean(pred != y_test)) * 100
        k = min(window_size, unlabeled.size)
        if strategy == "random":
            order = np.argsort(rng.uniform(size=unlabeled.size), kind="stable")
            chosen = unlabeled[order[:k]]
        elif select_fn is not None:
            chosen = np.asarray(select_fn(strategy, X, unlabeled, rf, k))
        else:
            forest = rf.forest if isinstance(rf, GpuForestModel) else Forest.from_sklearn(rf)
            if strategy == "uncertainty":
                from .uncertainty_sampling import select
                sel = select(state, unlabeled, forest, k)
            elif strategy == "density":
                from .density_weighting import select
                sel = select(state, unlabeled, forest, k, beta=beta)
            else:
                raise ValueError(f"unknown strategy {strategy!r}")
            chosen = sel.indices.cpu().numpy()
        res.labeled_history.append(chosen)
        res.accuracy.append(acc)
        labeled.extend(int(i) for i in chosen)
        unlabeled = np.setdiff1d(unlabeled, chosen, assume_unique=True)
        line = f"Iteration  {it}  -- accu =  {acc}"
        res.log.append(line)
        if verbose:
            print(line)
        it += 1
    return res
