"""Generate the committed golden fixtures under tests/golden/.

Runs ONLY in the build container (it reads data files of the read-only
reference at /root/reference and fits scikit-learn forests); the GPU box and
the test suite only load the resulting .npz/.json files.

    python tests/golden/make_golden.py

Inputs taken from the reference (data only, no source):
  * final_thesis/unlabeled_init.txt       2 x (784 features + label)
  * lal_direct_mllib_implementation/data/{checkerboard2x2,checkerboard4x4,
    rotated_checkerboard2x2}_train.txt    1000 x (2 features + label)
  * final_thesis/results/striatum_distDW_window_10_samples_5000.txt
                                          printed entropy lists (KAT for ent[v], T=10)
Expected outputs are computed by the CPU oracle (oracle/dal_oracle.py).
"""
from __future__ import annotations

import ast
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import dal_oracle as O  # noqa: E402

REF = "/root/reference"


def forest_arrays(f: O.OracleForest, prefix="forest_"):
    return {prefix + k: getattr(f, k) for k in
            ("feature", "threshold", "left", "right", "value", "roots")}


def fit_rf(X, y, n_trees=10, seed=0):
    from sklearn.ensemble import RandomForestClassifier
    rf = RandomForestClassifier(n_estimators=n_trees, max_depth=4, max_features="sqrt",
                                bootstrap=True, random_state=seed)
    rf.fit(X, y)
    return rf


def check_votes_vs_sklearn(rf, forest, X):
    per_tree = np.stack([est.predict(X.astype(np.float32)) for est in rf.estimators_])
    classes = rf.classes_
    hard = (classes[per_tree.astype(np.int64)] == 1).astype(np.int32).sum(axis=0)
    v = O.votes(forest, X)
    assert np.array_equal(hard, v), "oracle votes disagree with sklearn per-tree predict"


def selections(prefix, X, unl, forest, ks, excluded=None, density=None):
    out = {}
    for strat in O.STRATEGIES:
        for k in ks:
            sc, si, ss = O.uncertainty_select(X, unl, forest, k, strat)
            out[f"{prefix}us_{strat}_k{k}_idx"] = si
            out[f"{prefix}us_{strat}_k{k}_scores"] = ss
        out[f"{prefix}us_{strat}_scores"] = sc
    for k in ks:
        sc, si, ss = O.density_select(X, unl, forest, k, 1.0, excluded, density)
        out[f"{prefix}dw_k{k}_idx"] = si
        out[f"{prefix}dw_k{k}_scores"] = ss
    out[f"{prefix}dw_scores"] = sc
    return out


def kat_entropy():
    path = os.path.join(REF, "final_thesis/results/striatum_distDW_window_10_samples_5000.txt")
    vals = set()
    lines = []
    with open(path) as fh:
        for ln, line in enumerate(fh, 1):
            line = line.strip()
            if line.startswith("[") and "(" not in line and line.endswith("]"):
                items = ast.literal_eval(line.replace("nan", "None"))
                for x in items:
                    if x is not None:
                        vals.add(repr(float(x)))
                lines.append(ln)
    return {"source": "final_thesis/results/striatum_distDW_window_10_samples_5000.txt",
            "lines": lines, "T": 10, "values_repr": sorted(vals)}


def kat_topk_lists():
    """(idx, score) lists printed by density_weighting.py:170; used for
    order properties (descending, -0.0 ties)."""
    path = os.path.join(REF, "final_thesis/results/striatum_distDW_window_10_samples_5000.txt")
    out = []
    with open(path) as fh:
        for ln, line in enumerate(fh, 1):
            line = line.strip()
            if line.startswith("[("):
                items = ast.literal_eval(line.replace("nan", "None"))
                out.append({"line": ln, "pairs": [[int(i), (None if s is None else repr(float(s)))]
                                                  for i, s in items]})
    return out


def main():
    rng = np.random.default_rng(1234)

    # ---- LUTs + KAT ----------------------------------------------------
    for T in (10, 50, 100):
        np.savez(os.path.join(HERE, f"lut_T{T}.npz"), lc=O.lut_least_confidence(T),
                 mg=O.lut_margin(T), ent=O.lut_entropy(T))
    kat = kat_entropy()
    kat["topk_lists"] = kat_topk_lists()
    with open(os.path.join(HERE, "kat_dw_log_T10.json"), "w") as fh:
        json.dump(kat, fh, indent=1)

    # ---- config 1: unlabeled_init.txt (2 x 784) -------------------------
    raw = np.loadtxt(os.path.join(REF, "final_thesis/unlabeled_init.txt"))
    X = raw[:, :-1].astype(np.float32)
    y = raw[:, -1].astype(np.int64)
    rf = fit_rf(X, y, 10, 0)
    f = O.forest_from_sklearn(rf)
    check_votes_vs_sklearn(rf, f, X)
    unl = np.arange(2)
    d = O.density_canonical(X, [])
    dg = O.density_gram(X, [])
    out = {"X": X, "y": y, "unlabeled": unl, "votes": O.votes(f, X),
           "density": d, "density_gram": dg, **forest_arrays(f)}
    out.update(selections("", X, unl, f, (1, 2), excluded=[], density=d))
    np.savez_compressed(os.path.join(HERE, "unlabeled_init.npz"), **out)

    # ---- checkerboards (1000 x 2) --------------------------------------
    for name in ("checkerboard2x2", "checkerboard4x4", "rotated_checkerboard2x2"):
        raw = np.loadtxt(os.path.join(REF, f"lal_direct_mllib_implementation/data/{name}_train.txt"))
        X = raw[:, :-1].astype(np.float32)
        y = raw[:, -1].astype(np.int64)
        out = {"X": X, "y": y}
        E = np.arange(10)  # L0 = range(window_size), density_weighting.py:89
        d = O.density_canonical(X, E)
        out["excluded"] = E
        out["density"] = d
        out["density_gram"] = O.density_gram(X, E)
        for it, n_lab in (("it1_", 10), ("it5_", 50)):
            lab = np.arange(n_lab)
            unl = np.arange(n_lab, X.shape[0])
            yl = y[lab]
            if len(np.unique(yl)) == 1:
                # degenerate first iteration: all-one-class forest -> heavy ties
                pass
            rf = fit_rf(X[lab], yl, 10, 0)
            f = O.forest_from_sklearn(rf)
            check_votes_vs_sklearn(rf, f, X)
            out[it + "unlabeled"] = unl
            out[it + "votes"] = O.votes(f, X)
            out.update(forest_arrays(f, it + "forest_"))
            out.update(selections(it, X, unl, f, (1, 10), excluded=E, density=d))
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)

    # ---- synthetic pools ------------------------------------------------
    for (n, D, T, dist) in ((512, 64, 10, "uniform"), (4096, 256, 10, "uniform"),
                            (1500, 30, 100, "normal")):
        X = O.synthetic_pool(n, D, seed=0, dist=dist)
        f = O.synthetic_forest(T, 4, D, seed=1, dist=dist)
        E = np.arange(10)
        unl = np.arange(10, n)
        d = O.density_canonical(X, E)
        out = {"X": X, "excluded": E, "unlabeled": unl, "votes": O.votes(f, X),
               "density": d, "density_gram": O.density_gram(X, E), **forest_arrays(f)}
        out.update(selections("", X, unl, f, (1, 10, 100), excluded=E, density=d))
        L = np.arange(64)
        m, a = O.max_cosine(X, L)
        out["maxcos_labeled"] = L
        out["maxcos"] = m
        out["maxcos_arg"] = a
        di, ds = O.diversity_select(X, L, 32, candidates=np.arange(64, n))
        out["div_k32_idx"] = di
        out["div_k32_scores"] = ds
        np.savez_compressed(os.path.join(HERE, f"synthetic_{n}x{D}_T{T}.npz"), **out)

    # ---- standalone similarity kernels (D > 256 exercises K-slicing) ---
    X = O.synthetic_pool(96, 500, seed=3)
    i, j, v = O.column_similarities(X)
    np.savez_compressed(os.path.join(HERE, "similarity_96x500.npz"), X=X,
                        entries=O.cosine_entries(X), ci=i.astype(np.int32),
                        cj=j.astype(np.int32), cv=v)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
