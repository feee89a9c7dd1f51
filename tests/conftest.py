"""Test configuration.

``-m "not gpu"``: oracle vs golden fixtures, host logic, C-ABI exports,
multi-process (gloo) orchestration -- runs without a GPU.
``-m gpu``: parity of the HIP kernels (through the C ABI) against the oracle
and the committed golden fixtures; needs an MI355X and a built libdal.so.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "distributed-active-learning_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libdal.so")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_forest(g, prefix="forest_"):
    from oracle.dal_oracle import OracleForest

    return OracleForest(**{k: g[prefix + k] for k in
                           ("feature", "threshold", "left", "right", "value", "roots")})


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dal import _lib

    _lib.load()  # fails loudly if libdal.so is missing
    return torch.device("cuda:0")
