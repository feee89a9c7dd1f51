"""Which summation model does v_mfma_f32_16x16x32_f16 follow?  Random and
crafted 16x16x32 tiles (fp16 A, B; fp32 C) through scripts/libmfma_probe.so,
every output element compared bit for bit with candidate models:

  exact1   the 32 products and C summed exactly, rounded once (RNE)
  seqk     fp32 fmaf chain over k = 0..31 starting from C
  seqc     products summed exactly, then + C in fp32 ... (= exact1 on C = 0)
  grpG     exact sums of G consecutive products, fp32 chain over the groups from C

usage: python scripts/mfma_probe.py [cases]"""
import ctypes
import os
import sys
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    lib = ctypes.CDLL(os.path.join(HERE, "libmfma_probe.so"))
    p = ctypes.c_void_p
    lib.mfma_probe.argtypes = [p, p, p, p]
    return lib


def run(lib, A, B, C):
    """A [16, 32] fp16, B [16 cols, 32] fp16, C [16, 16] fp32 -> D [16, 16] fp32."""
    a = np.ascontiguousarray(A.astype(np.float16)).view(np.uint16)
    b = np.ascontiguousarray(B.astype(np.float16)).view(np.uint16)
    c = np.ascontiguousarray(C.astype(np.float32))
    d = np.zeros((16, 16), dtype=np.float32)
    rc = lib.mfma_probe(a.ctypes.data, b.ctypes.data, c.ctypes.data, d.ctypes.data)
    assert rc == 0
    return d


def f32(x: Fraction) -> np.float32:
    """Round an exact rational to fp32 (RNE) through fp64 pieces (exact enough:
    the fp64 of a Fraction is correctly rounded, and a double -> float RNE
    double rounding is avoided by checking the tie case exactly)."""
    d = float(x)  # correctly rounded to fp64
    f = np.float32(d)
    # fix double rounding: compare the exact distance to the two fp32 neighbours
    lo = np.nextafter(f, np.float32(-np.inf))
    hi = np.nextafter(f, np.float32(np.inf))
    best = f
    for cand in (lo, hi):
        if abs(Fraction(float(cand)) - x) < abs(Fraction(float(best)) - x):
            best = cand
        elif abs(Fraction(float(cand)) - x) == abs(Fraction(float(best)) - x):
            if (int(np.float32(cand).view(np.uint32)) & 1) == 0:
                best = cand
    return np.float32(best)


def models(a_row, b_col, c):
    prods = [Fraction(float(x)) * Fraction(float(y)) for x, y in zip(a_row, b_col)]
    C = Fraction(float(c))
    R = lambda x: Fraction(float(f32(x)))  # noqa: E731  (round to fp32, back to exact)
    out = {}
    out["exact1"] = sum(prods, C)
    acc = C
    for p in prods:
        acc = R(acc + p)
    out["seqk"] = acc
    for G in (4, 8, 16):
        g = [sum(prods[i:i + G], Fraction(0)) for i in range(0, 32, G)]
        acc = C
        for v in g:
            acc = R(acc + v)
        out[f"grp{G}_seqC"] = acc
        acc = R(g[0])
        for v in g[1:]:
            acc = R(acc + v)
        out[f"grp{G}_seq_thenC"] = R(acc + C)
        if G == 8:
            out["grp8_tree_thenC"] = R(R(R(g[0] + g[1]) + R(g[2] + g[3])) + C)
            out["grp8_tree_C"] = R(R(R(g[0] + g[1]) + R(g[2] + g[3]) ) + C)
            out["grp8_roundeach_exactsum_C"] = R(R(g[0]) + R(g[1]) + R(g[2]) + R(g[3]) + C)
            out["grp8_exact_pairs"] = R(R(g[0] + g[1] + C) + R(g[2] + g[3]))
    out["prods_then_c"] = R(R(sum(prods, Fraction(0))) + C)
    return {k: np.float32(float(v)) for k, v in out.items()}


def random_case(rng, kind):
    if kind == "uniform":
        A = rng.uniform(-1, 1, (16, 32)) * 2048
        B = rng.uniform(-1, 1, (16, 32)) * 2048
    elif kind == "wide":  # products over a wide exponent range
        A = rng.choice([-1, 1], (16, 32)) * 2.0 ** rng.integers(-14, 15, (16, 32)) * rng.uniform(1, 2, (16, 32))
        B = rng.choice([-1, 1], (16, 32)) * 2.0 ** rng.integers(-14, 15, (16, 32)) * rng.uniform(1, 2, (16, 32))
    else:  # the Gram's operand: H = fp16(2^12 u), u >= 0
        A = rng.random((16, 32)) * 4096
        B = rng.random((16, 32)) * 4096
    A = A.astype(np.float16).astype(np.float64)
    B = B.astype(np.float16).astype(np.float64)
    C = (rng.uniform(-1, 1, (16, 16)) * 2.0 ** rng.integers(0, 30, (16, 16))).astype(np.float32)
    if kind == "gram":
        C = np.abs(C)
    return A, B, C


def main():
    lib = load()
    n_cases = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    rng = np.random.default_rng(0)
    hits = {}
    total = 0
    miss_example = None
    for t in range(n_cases):
        kind = ("uniform", "wide", "gram")[t % 3]
        A, B, C = random_case(rng, kind)
        D = run(lib, A, B, C)
        for i in range(16):
            for j in range(16):
                m = models(A[i], B[j], C[i, j])
                total += 1
                for name, v in m.items():
                    if np.float32(v).view(np.uint32) == np.float32(D[i, j]).view(np.uint32):
                        hits[name] = hits.get(name, 0) + 1
                if miss_example is None and np.float32(m["grp8_seqC"]) != D[i, j]:
                    miss_example = (kind, float(D[i, j]), {k: float(v) for k, v in m.items()})
    print(f"{total} outputs; bit-exact matches per model:")
    for name in sorted(hits, key=lambda k: -hits[k]):
        print(f"  {name:28s} {hits[name]}")
    print("first grp8_seqC miss:", miss_example)
    # crafted, on the diagonal: row r of A against column r of B
    A = np.zeros((16, 32))
    B = np.zeros((16, 32))
    trip = [(0, 3, 5), (1, 10, 18), (2, 17, 31), (3, 24, 12), (7, 20, 0), (9, 8, 15), (16, 17, 18), (31, 0, 15),
            (8, 16, 24), (24, 16, 8), (4, 12, 20), (30, 22, 14)]
    for r, (i, j, m) in enumerate(trip):
        A[r, [i, j, m]] = [4096, 1, -4096]
        B[r, [i, j, m]] = [4096, 1, 4096]
    D = run(lib, A, B, np.zeros((16, 16), np.float32))
    for r, tr in enumerate(trip):
        print(f"  [2^24 @k{tr[0]}, 1 @k{tr[1]}, -2^24 @k{tr[2]}] -> {float(D[r, r])} (exact 1)")
    C = np.zeros((16, 16), np.float32)
    C[0, 0] = 2.0 ** 24
    A = np.zeros((16, 32))
    B = np.zeros((16, 32))
    A[0, :] = 1
    B[0, :] = 1
    D = run(lib, A, B, C)
    print("C = 2^24 + 32 products of 1 (exact 2^24 + 32):", float(D[0, 0]) - 2 ** 24)


if __name__ == "__main__":
    main()
