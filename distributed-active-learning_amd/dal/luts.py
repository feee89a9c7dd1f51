"""fp64 score look-up tables indexed by the integer vote count v in {0..T}.

The reference evaluates these per row in a Python lambda on float64; since v
takes only T+1 values, the product evaluates the same Python float
expressions once per v on the host and the GPU indexes the table.  Keeping the
reference's exact operation order matters: at T=100, 8 of the 50 symmetric vote
pairs of the least-confidence score do NOT tie in fp64 (e.g. v=41 ->
0.09000000000000008, v=59 -> 0.08999999999999997).

  least_confidence  abs(0.5 - (1 - (v/T)))          uncertainty_sampling.py:98,
                                                    active_learner.py:197   (ascending)
  margin            abs((v/T) - (1 - (v/T)))        binary margin            (ascending)
  entropy           -(1-(v/T)) * log2(1-(v/T))      density_weighting.py:148 (descending)
                    v=0 -> -0.0, v=T -> NaN (0 * -inf)
"""
from __future__ import annotations

import math

import numpy as np

STRATEGIES = ("least_confidence", "margin", "entropy")
ASCENDING = {"least_confidence": True, "margin": True, "entropy": False}


def _log2(p: float) -> float:
    # log(x)/log(2) reproduces the reference's printed value for v=1, T=10
    # (0.13680278410054497, results/striatum_distDW_window_10_samples_5000.txt);
    # numpy 2.x log2 differs by one ulp there.
    return math.log(p) / math.log(2)


def lut(strategy: str, n_trees: int) -> np.ndarray:
    T = int(n_trees)
    if T < 1:
        raise ValueError("n_trees must be >= 1")
    if strategy == "least_confidence":
        vals = [abs(0.5 - (1 - (v / T))) for v in range(T + 1)]
    elif strategy == "margin":
        vals = [abs((v / T) - (1 - (v / T))) for v in range(T + 1)]
    elif strategy == "entropy":
        vals = []
        for v in range(T + 1):
            p0 = 1 - (v / T)
            vals.append(-(p0) * _log2(p0) if p0 > 0.0 else float("nan"))
    else:
        raise ValueError(f"unknown strategy {strategy!r}; expected one of {STRATEGIES}")
    return np.array(vals, dtype=np.float64)
