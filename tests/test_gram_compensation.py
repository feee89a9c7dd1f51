"""The compensated symmetric Gram's algebra (csrc/gram_sym.hip), restated in
NumPy on exact integers (CPU only): over super-block pairs taken by the
orientation rule, the H-only taker side gives the row sums of H_P (H_Q +
L_Q)^T (the MFMA kernel); the closed form of dal_gram_sym_residual --
<L_r, R_B> (the taker side's remainder) + <u~_r, C_B> (the column sums of
every pair that takes r's super block) with R_B / C_B the parity-class prefix
sums of the super blocks' u~ sums that csym_scan_kernel forms -- completes
every row to sum_j <u~_r, u~_j> exactly.  Reference:
density_weighting.py:67-75,157-161."""
import numpy as np
import pytest

SB = 512


def takes(P, Q):
    return Q == P or (Q > P and (P + Q) % 2 == 0) or (Q < P and (P + Q) % 2 == 1)


def residual(H, L, nsb):
    U = H + L
    D = H.shape[1]
    sig_u = np.array([U[q * SB:(q + 1) * SB].sum(0) for q in range(nsb)])
    tot = [sig_u[0::2].sum(0), sig_u[1::2].sum(0)]
    e = [np.zeros(D, dtype=np.int64) for _ in range(2)]
    res = np.zeros(H.shape[0], dtype=np.int64)
    for q in range(nsb):
        b = q & 1
        R = tot[b] - e[b] + e[1 - b]          # sum of u~ over the super blocks q takes
        C = e[b] + tot[1 - b] - e[1 - b]      # sum of u~ over the other super blocks taking q
        rows = slice(q * SB, (q + 1) * SB)
        res[rows] = L[rows] @ R + U[rows] @ C
        e[b] = e[b] + sig_u[q]
    return res


@pytest.mark.parametrize("nsb,D,seed", [(1, 4, 0), (2, 8, 1), (7, 8, 2), (10, 3, 3)])
def test_compensated_sym_gram_completes_every_row(nsb, D, seed):
    rng = np.random.default_rng(seed)
    n = nsb * SB
    H = rng.integers(-2048, 2048, (n, D)).astype(np.int64)
    L = rng.integers(-2, 3, (n, D)).astype(np.int64)
    H[rng.random(n) < 0.05] = 0  # excluded / padding rows are zero rows
    U = H + L
    acc = np.zeros(n, dtype=np.int64)
    for P in range(nsb):
        for Q in range(nsb):
            if not takes(P, Q):
                continue
            T = H[P * SB:(P + 1) * SB] @ U[Q * SB:(Q + 1) * SB].T
            acc[P * SB:(P + 1) * SB] += T.sum(axis=1)  # row sums only (the kernel)
    full = U @ U.sum(axis=0)
    assert np.array_equal(acc + residual(H, L, nsb), full)
    if nsb > 1:
        assert not np.array_equal(acc, full)  # the remainder is not negligible in this test


def test_every_unordered_pair_taken_once():
    for nsb in (1, 2, 5, 8):
        for P in range(nsb):
            for Q in range(nsb):
                assert takes(P, Q) + (takes(Q, P) if P != Q else 0) == 1
