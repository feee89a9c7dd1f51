"""Product LUTs vs oracle; the C ABI library exports every declared symbol
and validates arguments on the host.  CPU only (no kernel launches)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO
from dal import _lib, luts
from oracle import dal_oracle as O


@pytest.mark.parametrize("T", [1, 2, 3, 10, 50, 100, 2000])
@pytest.mark.parametrize("strategy", luts.STRATEGIES)
def test_product_luts_equal_oracle(T, strategy):
    assert np.array_equal(luts.lut(strategy, T), O.lut(strategy, T), equal_nan=True)
    assert np.array_equal(np.signbit(luts.lut(strategy, T)), np.signbit(O.lut(strategy, T)))


def header_functions():
    src = open(os.path.join(REPO, "include", "dal.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dal_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


def test_host_helpers():
    lib = _lib.load()
    assert lib.dal_abi_version() == 10
    assert lib.dal_pad_rows(1) == 512 and lib.dal_pad_rows(100000) == 100352
    assert [lib.dal_pad_features(d) for d in (1, 30, 33, 64, 65, 128, 129, 256, 500, 784)] == \
        [32, 32, 64, 64, 128, 128, 256, 256, 512, 1024]
    assert lib.dal_status_string(-2).decode().startswith("shape")
    b = lib.dal_density_error_bound(100000)
    assert 1.0 < b < 10.0  # ~3.1e-5 * N
    bsym = lib.dal_density_error_bound_sym(100000)
    assert b < bsym < 30.0  # ~2.45e-4 * N (chains of <= 2,048 fp32 adds, conservative MFMA model)
    # row-side chain by slice width (one chain per row tile at KS
    # 64 / 128 sums 2,048 products between folds, KS 32 1,024)
    u = 2.0 ** -23
    c = 1.0 + 1.0 / 256.0

    def expect(chain, n):
        g = (chain + 5) * u / (1 - (chain + 5) * u)
        return (g * c + 5 * 2.0 ** -22 + 1e-10) * n + 1e-9

    for d_pad, chain in ((32, 1024), (64, 2048), (128, 2048), (256, 2048), (0, 2048)):
        got = lib.dal_density_error_bound_sym_d(100000, d_pad)
        assert abs(got - expect(chain, 100000)) <= 1e-12 * got, (d_pad, got)
    assert lib.dal_density_error_bound_sym_d(100000, 0) == bsym
    assert lib.dal_density_error_bound_sym_d(100000, 32) < bsym
    # sigma~ per super block, then R_B and C_B per requested super block
    assert lib.dal_gram_sym_residual_workspace_bytes(392, 392, 64) == 196 * 64 * 8 + 2 * 196 * 64 * 8
    assert lib.dal_gram_sym_residual_workspace_bytes(0, 2, 64) == 0
    assert lib.dal_split_f16_halves(512, 64) == 512 * 128
    assert lib.dal_topk_workspace_bytes(1 << 21, 1000) > 0


def test_host_argument_validation_without_gpu():
    lib = _lib.load()
    # null pointers -> DAL_ERR_ARG before any HIP call
    assert lib.dal_normalize_rows(None, 10, 4, 4, None, 512, 32, None, None, None, None) == -1
    assert lib.dal_gram_rowsum(None, 256, None, 512, 64, 64, None, 0, None) == -1
    assert lib.dal_topk(None, 10, 1, 0, None, 0, None, None, None) == -1
    # bad shapes -> DAL_ERR_SHAPE
    p = ctypes.c_void_p(256)
    assert lib.dal_gram_rowsum(p, 100, p, 512, 64, 64, p, 0, None) == -2
    assert lib.dal_gram_rowsum(p, 256, p, 500, 64, 64, p, 0, None) == -2
    assert lib.dal_gram_rowsum(p, 256, p, 512, 48, 64, p, 0, None) == -2
    assert lib.dal_gram_rowsum_sym_skip(None, 0, 2, p, 0, 0, 2, 0, 0, 2, 64, p, 0, None) == -1
    assert lib.dal_gram_rowsum_sym_skip(p, 0, 3, p, 0, 0, 2, 0, 0, 4, 64, p, 0, None) == -2  # odd row blocks
    assert lib.dal_gram_rowsum_sym_skip(p, 0, 2, p, 0, 0, 6, 0, 0, 4, 64, p, 0, None) == -2  # j_hi > nb_active
    assert lib.dal_gram_rowsum_sym_skip(p, 0, 2, p, 0, 0, 2, 0, 0, 2, 48, p, 0, None) == -2  # d_pad
    assert lib.dal_gram_sym_residual(None, 2, 0, 2, 64, p, p, 1 << 20, None) == -1
    assert lib.dal_gram_sym_residual(p, 2, 1, 2, 64, p, p, 1 << 20, None) == -2   # odd block
    assert lib.dal_gram_sym_residual(p, 2, 0, 2, 64, p, p, 16, None) == -2        # workspace too small
    assert lib.dal_split_f16(None, 512, 64, 64, None, None) == -1
    assert lib.dal_split_f16(p, 500, 64, 64, p, None) == -2
    assert lib.dal_topk(p, 10, 11, 0, p, 1 << 20, p, p, None) == -2
    assert lib.dal_topk(p, 100000, 9000, 0, p, 1 << 30, p, p, None) == -5
    assert lib.dal_forest_score(p, 10, 4, 4, p, p, 3, 17, p, None, 0, 0.0, None, 1.0, 0, p, p, p,
                                None, None) == -3


def test_blocked_pool_rule_without_gpu():
    """ABI v9: the blocked K2 path applies when a tile's runs -- the forest's
    node count bounds its distinct features -- number <= 256 and fit 96 KiB of
    LDS with the forest, and a wave's partial vote fits 8 bits; the copy's
    size is whole 64-row tiles; bad arguments are rejected before any HIP call."""
    lib = _lib.load()
    assert lib.dal_forest_blocked_rows(256, 10, 4) == 64     # config 4 (150 runs)
    assert lib.dal_forest_blocked_rows(256, 100, 4) == 64    # config 4 at T = 100 (256 runs)
    assert lib.dal_forest_blocked_rows(64, 10, 4) == 64      # config 2
    assert lib.dal_forest_blocked_rows(30, 100, 4) == 64     # config 3
    assert lib.dal_forest_blocked_rows(512, 100, 4) == 0     # 512 runs
    assert lib.dal_forest_blocked_rows(300, 100, 8) == 0     # a 204-KB forest
    assert lib.dal_forest_blocked_rows(20, 1021, 1) == 0     # partial votes past 8 bits
    assert lib.dal_forest_blocked_rows(20, 1020, 1) == 64
    assert lib.dal_forest_blocked_rows(0, 10, 4) == 0 and lib.dal_forest_blocked_rows(256, 10, 17) == 0
    assert lib.dal_pool_blocked_floats(1, 256) == 64 * 256 and lib.dal_pool_blocked_floats(128, 3) == 128 * 3
    assert lib.dal_pool_blocked_floats(0, 8) == 0 and lib.dal_pool_blocked_floats(10, 0) == -1
    p = ctypes.c_void_p(256)
    assert lib.dal_pool_blocked(None, 10, 4, 4, p, None) == -1
    assert lib.dal_pool_blocked(p, 10, 4, 3, p, None) == -2
    assert lib.dal_pool_blocked(p, 0, 4, 4, p, None) == 0  # nothing to copy: no launch
    odd = ctypes.c_void_p(264)  # xb and fprep must be 16-B aligned
    assert lib.dal_forest_score_blocked(p, odd, None, 10, 256, 256, p, p, 10, 4, p, None, 0, 0.0, None, 1.0, 0,
                                        p, p, p, None, None) == -1
    assert lib.dal_forest_score_blocked(p, p, odd, 10, 256, 256, p, p, 10, 4, p, None, 0, 0.0, None, 1.0, 0,
                                        p, p, p, None, None) == -1


def test_forest_prep_rule_without_gpu():
    """ABI v10: the prepared forest is a 16-B header and the blocked kernel's
    LDS forest region (nodes int2, leaves rounded to 4 B, the u16 feature list
    for at most min(nodes, d) features), padded to 16 B; 0 bytes where the
    blocked path does not apply.  Bad arguments are rejected before any HIP call."""
    lib = _lib.load()

    def expect(d, t, depth):
        nn = t * (2 ** depth - 1)
        fu = min(nn, d)
        pay = nn * 8 + -(-t * 2 ** depth // 4) * 4 + -(-fu // 2) * 4
        return 16 + -(-pay // 16) * 16

    for d, t in ((256, 10), (256, 100), (64, 10), (30, 100)):
        assert lib.dal_forest_prep_bytes(d, t, 4) == expect(d, t, 4), (d, t)
    assert lib.dal_forest_prep_bytes(512, 100, 4) == 0 and lib.dal_forest_prep_bytes(0, 10, 4) == 0
    assert lib.dal_forest_prep_bytes(256, 10, 17) == 0
    p = ctypes.c_void_p(256)
    odd = ctypes.c_void_p(264)
    nb = lib.dal_forest_prep_bytes(256, 10, 4)
    assert lib.dal_forest_prepare(None, p, 10, 4, 256, p, nb, None) == -1
    assert lib.dal_forest_prepare(p, p, 10, 4, 256, odd, nb, None) == -1
    assert lib.dal_forest_prepare(p, p, 10, 4, 256, p, nb - 16, None) == -2
    assert lib.dal_forest_prepare(p, p, 10, 4, 0, p, nb, None) == -2
    assert lib.dal_forest_prepare(p, p, 10, 17, 256, p, nb, None) == -3
    assert lib.dal_forest_prepare(p, p, 100, 4, 512, p, 1 << 20, None) == -3  # not blocked: 512 runs


def test_merge_and_mark_count_validation_without_gpu():
    """ABI v4 entry points reject bad arguments before any HIP call."""
    lib = _lib.load()
    p = ctypes.c_void_p(256)
    assert lib.dal_topk_merge_workspace_bytes(8, 1000) == 8 * 1000 * 16 + 1000 * 16
    assert lib.dal_topk_merge_workspace_bytes(8, 100) == 0  # one launch, no workspace
    assert lib.dal_topk_merge_workspace_bytes(0, 100) == 0
    assert lib.dal_topk_merge(None, 2, 301, 100, p, 1 << 20, p, p, None, p, None) == -1
    assert lib.dal_topk_merge(p, 2, 300, 100, p, 1 << 20, p, p, None, p, None) == -2  # no room for status
    assert lib.dal_topk_merge(p, 0, 301, 100, p, 1 << 20, p, p, None, p, None) == -2
    assert lib.dal_topk_merge(p, 9, 3001, 1000, p, 1 << 20, p, p, None, p, None) == -5  # > DAL_SORT_CAP
    assert lib.dal_topk_merge(p, 5, 3001, 1000, p, 16, p, p, None, p, None) == -5  # workspace too small
    assert lib.dal_topk_merge(p, 5, 3001, 1000, None, 1 << 30, p, p, None, p, None) == -1  # needs one
    assert lib.dal_mark_rows_count(None, 10, 0, 10, 1, p, p, None) == -1
    assert lib.dal_mark_rows_count(p, 10, 0, 10, 1, p, None, None) == -1
    assert lib.dal_mark_rows_count(p, -1, 0, 10, 1, p, p, None) == -2


def test_maxcos_unit_bound_and_validation_without_gpu():
    """ABI v7: the folded-operand max-cosine's bound (one fp16 rounding of
    the unit labeled rows dominates: ~2^-11) and argument checks before any
    HIP call."""
    lib = _lib.load()
    p = ctypes.c_void_p(256)
    for d in (64, 128, 256):
        b, b16 = lib.dal_maxcos_unit_error_bound(d), lib.dal_maxcos_error_bound(d)
        assert 2.0 ** -11 < b < 2.0 ** -11 * 1.2 and b > 10 * b16
    assert lib.dal_max_cosine_unit(None, 10, 128, p, 256, p, p, None) == -1
    assert lib.dal_max_cosine_unit(p, 10, 96, p, 256, p, p, None) == -2      # d not 64/128/256
    assert lib.dal_max_cosine_unit(p, 10, 128, p, 300, p, p, None) == -2     # m_pad off the granule
    assert lib.dal_max_cosine_unit(p, 10, 128, p, 8192, p, p, None) == -2    # > 4096 labeled rows
    assert lib.dal_max_cosine_unit(ctypes.c_void_p(264), 10, 128, p, 256, p, p, None) == -2  # unaligned
    assert lib.dal_unit_rows_f16(None, 4, 256, 128, 128, p, p, None) == -1
    assert lib.dal_unit_rows_f16(p, 4, 2, 128, 128, p, p, None) == -2        # m_pad < m
