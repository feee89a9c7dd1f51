"""ctypes binding of libdal.so (the C ABI declared in include/dal.h).

The library is built in-tree (``make -C distributed-active-learning_amd/csrc``
or ``__graft_entry__.build()``) and loaded from this directory.  There is no
fallback: if the library is missing or a call fails, this module raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_double, c_int, c_int32, c_int64, c_size_t, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdal.so")

# constants mirrored from include/dal.h
DAL_OK = 0
DAL_FLAG_ZERO_NORM = 1
DAL_FLAG_CAND_OVERFLOW = 2
DAL_FLAG_RF_SPLITS = 4
DAL_FLAG_SAMPLE_MISS = 8
DAL_ROW_CANDIDATE = 1
DAL_ROW_EXCLUDED = 2
DAL_DENSITY_NONE = 0
DAL_DENSITY_FIXED = 1
DAL_DENSITY_EXACT = 2
DAL_ASCENDING = 0
DAL_DESCENDING = 1
DAL_KEY_NAN = 0xFFFFFFFFFFFFFFFE
DAL_KEY_NONE = 0xFFFFFFFFFFFFFFFF
DAL_FIXED_SCALE = 4294967296.0
DAL_ROW_GRANULE = 512
DAL_CANON_CHUNK = 256
DAL_MAX_TREE_DEPTH = 16
DAL_SORT_CAP = 8192
DAL_SORT_CAP_PAYLOAD = 4096
DAL_STEP_RESET_STATUS = 1
DAL_STEP_WS_CLEAN = 2
DAL_STEP_KEEP_GROUPS = 4
DAL_STEP_SELECT_ONLY = 8
DAL_RF_MAX_SPLITS = 255
DAL_RF_MAX_SPLIT_SAMPLE = 16384
DAL_RF_MAX_DEPTH = 10
DAL_RF_SPLIT_LDS_BYTES = 163840

# name -> (restype, argtypes); every symbol of include/dal.h
SIGNATURES = {
    "dal_status_string": (ctypes.c_char_p, [c_int]),
    "dal_abi_version": (c_int, []),
    "dal_pad_rows": (c_int64, [c_int64]),
    "dal_pad_features": (c_int64, [c_int64]),
    "dal_density_error_bound": (c_double, [c_int64]),
    "dal_normalize_rows": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_int64, c_int64,
                                   c_void_p, c_void_p, c_void_p, c_void_p]),
    "dal_mark_rows_count": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p]),
    "dal_mark_rows": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int, c_void_p, c_void_p]),
    "dal_canon_colsum_partials": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p,
                                          c_void_p, c_void_p]),
    "dal_canon_colsum_reduce": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
    "dal_gram_rowsum": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int64, c_void_p,
                                c_int, c_void_p]),
    "dal_split_f16_halves": (c_int64, [c_int64, c_int64]),
    "dal_split_f16": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p]),
    "dal_prep_split": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_int64, c_int64,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "dal_density_error_bound_sym": (c_double, [c_int64]),
    "dal_density_error_bound_sym_d": (c_double, [c_int64, c_int64]),
    "dal_gram_rowsum_sym": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64, c_int64,
                                    c_int64, c_int64, c_void_p, c_int, c_void_p]),
    "dal_gram_rowsum_sym_skip": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64, c_int64,
                                         c_int64, c_int64, c_int64, c_int64, c_void_p, c_int, c_void_p]),
    "dal_gram_sym_residual_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "dal_gram_sym_residual": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p, c_void_p,
                                      c_size_t, c_void_p]),
    "dal_forest_score": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_int32,
                                 c_int32, c_void_p, c_void_p, c_int, c_double, c_void_p, c_double,
                                 c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "dal_forest_blocked_rows": (c_int, [c_int64, c_int32, c_int32]),
    "dal_pool_blocked_floats": (c_int64, [c_int64, c_int64]),
    "dal_pool_blocked": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p]),
    "dal_forest_prep_bytes": (c_size_t, [c_int64, c_int32, c_int32]),
    "dal_forest_prepare": (c_int, [c_void_p, c_void_p, c_int32, c_int32, c_int64, c_void_p, c_size_t, c_void_p]),
    "dal_forest_score_blocked": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p,
                                         c_int32,
                                         c_int32, c_void_p, c_void_p, c_int, c_double, c_void_p, c_double,
                                         c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "dal_density_separable": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p]),
    "dal_topk_workspace_bytes": (c_size_t, [c_int64, c_int64]),
    "dal_topk": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_size_t, c_void_p, c_void_p,
                         c_void_p]),
    "dal_dw_select_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "dal_dw_select": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64,
                              c_void_p, c_double, c_void_p, c_int64, c_int64, c_void_p, c_void_p,
                              c_int64, c_int32, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p]),
    "dal_dw_step_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "dal_dw_step": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_int32, c_int32, c_void_p,
                            c_void_p, c_double, c_void_p, c_double, c_int64, c_void_p, c_void_p, c_int64, c_int64,
                            c_int32, ctypes.c_uint32, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "dal_dw_plan_create": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_int32, c_int32,
                                   c_void_p, c_void_p, c_double, c_void_p, c_void_p, c_double, c_int64, c_void_p,
                                   c_void_p, c_int64, c_int64, c_int32, c_void_p, c_size_t, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "dal_dw_plan_run": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "dal_dw_plan_launch": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "dal_dw_plan_destroy": (None, [c_void_p]),
    "dal_maxcos_label_rows_granule": (c_int64, [c_int64]),
    "dal_maxcos_error_bound": (c_double, [c_int64]),
    "dal_inv_norms_bf16": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p, c_void_p,
                                   c_void_p]),
    "dal_canon_unit_rows_bf16": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int, c_void_p, c_void_p]),
    "dal_max_cosine": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_void_p]),
    "dal_unit_rows_f16": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    "dal_maxcos_unit_error_bound": (c_double, [c_int64]),
    "dal_max_cosine_unit": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "dal_text_shape": (c_int, [c_void_p, c_size_t, c_int64, c_void_p, c_void_p]),
    "dal_parse_labeled_text": (c_int, [c_void_p, c_size_t, c_int64, c_int64, c_int, c_void_p, c_void_p, c_int]),
    "dal_maxcos_argmax_resolve": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_int64, c_void_p,
                                          c_void_p]),
    "dal_interval_keys_f32": (c_int, [c_void_p, c_int64, c_double, c_void_p, c_int, c_void_p,
                                      c_void_p, c_void_p]),
    "dal_maxcos_select_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "dal_maxcos_select": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p, c_int64,
                                  c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_size_t, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p]),
    "dal_topk_merge_workspace_bytes": (c_size_t, [c_int64, c_int64]),
    "dal_topk_merge": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_size_t, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p]),
    "dal_sort_pairs": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p,
                               c_void_p, c_void_p]),
    "dal_gram_entries": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p]),
    "dal_rf_find_splits": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_int64, c_int32, c_void_p,
                                   c_void_p, c_void_p, c_void_p]),
    "dal_rf_train_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int32, c_int32, c_int32, c_int32]),
    "dal_rf_train": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_int32,
                             c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_double, c_void_p,
                             c_void_p, c_void_p, c_size_t, c_void_p]),
}

_lib = None


class DalError(RuntimeError):
    pass


def load():
    """Load libdal.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DalError(
            f"{LIB_PATH} not found: build the HIP library first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != DAL_OK:
        msg = load().dal_status_string(rc).decode()
        raise DalError(f"{what} failed: {msg} (status {rc})")


def call(name: str, *args):
    """Call a status-returning entry point and raise on failure."""
    rc = getattr(load(), name)(*args)
    check(rc, name)
