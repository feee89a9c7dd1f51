"""Timing of GPU random-forest training (dal.random_forest.train_classifier)
against scikit-learn's fit on the host and the CPU oracle (MLlib 2.1
restatement), on AL-sized labeled sets.  usage: python scripts/rf_train_bench.py"""
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "distributed-active-learning_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dal.random_forest import bagging_inputs, train_classifier  # noqa: E402

dev = torch.device("cuda:0")
shapes = [(1000, 30, 10), (5000, 64, 10), (5000, 30, 100), (20000, 64, 10), (2000, 784, 10)]
for n, d, T in shapes:
    rng = np.random.default_rng(n + d)
    X = rng.random((n, d), dtype=np.float32)
    y = (X[:, : max(1, d // 8)].sum(axis=1) > d // 16).astype(np.int64)
    w, s = bagging_inputs(n, d, T, 4, seed=1)
    xd = torch.from_numpy(X).to(dev)
    for _ in range(3):
        train_classifier(xd, y, T, weights=w, feature_subsets=s, device=dev)
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        F = train_classifier(xd, y, T, weights=w, feature_subsets=s, device=dev)
    torch.cuda.synchronize()
    gpu_ms = (time.perf_counter() - t0) / reps * 1e3
    from sklearn.ensemble import RandomForestClassifier

    t0 = time.perf_counter()
    RandomForestClassifier(n_estimators=T, max_depth=4, max_features="sqrt", bootstrap=True,
                           random_state=0, n_jobs=-1).fit(X, y)
    sk_ms = (time.perf_counter() - t0) * 1e3
    line = f"n={n} d={d} T={T}: GPU train {gpu_ms:.2f} ms (incl. host draws + D2H of the forest); sklearn fit {sk_ms:.1f} ms"
    if n * T <= 50000:
        from oracle import rf_oracle as R

        t0 = time.perf_counter()
        R.train_classifier(X, y, w, s)
        line += f"; CPU oracle {1e3 * (time.perf_counter() - t0):.0f} ms"
    print(line, flush=True)
