"""ctypes binding of libcfk_als.so (include/als.h + include/als_host.h).

The library is the product: there is no Python or CPU fallback. If the shared library is missing, or a
HIP call fails, the caller gets an exception -- never silently different numbers.

torch is imported BEFORE the library is dlopen'ed: torch ships its own libamdhip64.so (same SONAME), and
loading it first makes our library bind to that one HIP runtime instead of a second copy.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede dlopen of libcfk_als.so; see module docstring)

_PKG = os.path.dirname(os.path.abspath(__file__))
# CFK_ALS_LIB: another build of the same library (tools/kbench.py A/B of two builds on one box)
LIB_PATH = os.environ.get("CFK_ALS_LIB") or os.path.join(_PKG, "build", "libcfk_als.so")
APP_PATH = os.path.join(_PKG, "build", "als_app")

ALS_OK = 0
SIDE_MOVIE = 0
SIDE_USER = 1
F32 = 0
F64 = 1

_STATUS = {
    1: "ALS_ERR_INVALID_ARGUMENT", 2: "ALS_ERR_UNSUPPORTED", 3: "ALS_ERR_DEVICE", 4: "ALS_ERR_OUT_OF_MEMORY",
    5: "ALS_ERR_STATE", 6: "ALS_ERR_IO", 7: "ALS_ERR_PARSE", 8: "ALS_ERR_DATA", 9: "ALS_ERR_INTEGRITY",
    10: "ALS_ERR_COMM",
}


class ALSError(RuntimeError):
    def __init__(self, status: int, fn: str, msg: str):
        super().__init__(f"{fn}: {_STATUS.get(status, status)}: {msg}")
        self.status = status


_lib = None

# (name, restype, argtypes) -- every symbol declared in include/als.h and include/als_host.h
_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_f = ctypes.c_float
_u64 = ctypes.c_uint64
_pi64 = ctypes.POINTER(ctypes.c_int64)
_pi32 = ctypes.POINTER(ctypes.c_int32)
_pi16 = ctypes.POINTER(ctypes.c_int16)
_pf = ctypes.POINTER(ctypes.c_float)
_pu8 = ctypes.POINTER(ctypes.c_uint8)
_pd = ctypes.POINTER(ctypes.c_double)
_ppv = ctypes.POINTER(ctypes.c_void_p)

SIGNATURES = [
    ("als_abi_version", _i, []),
    ("als_last_error", ctypes.c_char_p, []),
    ("als_build_source_sha256", ctypes.c_char_p, []),
    ("als_device_count", _i, [ctypes.POINTER(ctypes.c_int)]),
    ("als_engine_create", _i, [_i, _i, _i, _ppv]),
    ("als_engine_destroy", _i, [_vp]),
    ("als_engine_set_stream", _i, [_vp, _vp]),
    ("als_engine_use_default_stream", _i, [_vp]),
    ("als_factor_stride", _i, [_vp]),
    ("als_set_block", _i, [_vp, _i, _i64, _i64, _i64, _pi64, _pi32, _pi16]),
    ("als_set_block_coo", _i, [_vp, _i, _i64, _i64, _i64, _i64, _pi32, _pi32, _pi16]),
    ("als_alloc_factors", _i, [_vp, _i, _i64]),
    ("als_bind_factors", _i, [_vp, _i, _vp, _i64]),
    ("als_factors_device_ptr", _i, [_vp, _i, _ppv, _pi64]),
    ("als_write_factors", _i, [_vp, _i, _i64, _i64, _vp, _i64]),
    ("als_read_factors", _i, [_vp, _i, _i64, _i64, _vp, _i64]),
    ("als_solve_half", _i, [_vp, _i, _f]),
    ("als_set_chunks", _i, [_vp, _i, _i, _pi64]),
    ("als_solve_half_chunk", _i, [_vp, _i, _f, _i]),
    ("als_comm_unique_id", _i, [_vp, _i]),
    ("als_comm_init", _i, [_vp, _i, _i, _vp]),
    ("als_comm_init_group", _i, [_ppv, _i]),
    ("als_comm_info", _i, [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    ("als_allgather_shard", _i, [_vp, _i, _i64, _i64]),
    ("als_set_row_layout", _i, [_vp, _i, _i64, _i64]),
    ("als_comm_group_start", _i, []),
    ("als_comm_group_end", _i, []),
    ("als_comm_wait", _i, [_vp]),
    ("als_comm_set_timeout", _i, [_vp, _i64]),
    ("als_predict", _i, [_vp, _pi64, _i64, _pi64, _i64, _pf]),
    ("als_sq_error", _i, [_vp, _i, _pd, _pi64]),
    ("als_synchronize", _i, [_vp]),
    ("als_integrity_status", _i, [_vp, ctypes.POINTER(ctypes.c_uint32), _i]),
    ("als_set_timing", _i, [_vp, _i]),
    ("als_timing_collect", _i, [_vp, _i, _pd, _pd, _pi64]),
    ("als_debug_copy_partials", _i, [_vp, _vp, _i64, _pi64]),
    ("als_block_path", _i, [_vp, _i, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), _pi64, _pi64]),
    ("als_block_stats", _i, [_vp, _i, _pi64, _pi64, _pi64]),
    ("als_block_split_info", _i, [_vp, _i, _pi64]),
    # als_host.h
    ("als_dataset_load_netflix", _i, [ctypes.c_char_p, _ppv]),
    ("als_dataset_from_ratings", _i, [_i64, _pi32, _pi32, _pi16, _ppv]),
    ("als_dataset_synthetic_netflix", _i, [_i64, _i64, _i64, _u64, _i, _ppv]),
    ("als_dataset_synthetic_powerlaw", _i, [_i64, _i64, _i64, _u64, _i, _ppv]),
    ("als_dataset_synthetic_powerlaw_shard", _i, [_i64, _i64, _i64, _u64, _i, _i, _i, _ppv]),
    ("als_dataset_synthetic_netflix_shard", _i, [_i64, _i64, _i64, _u64, _i, _i, _i, _ppv]),
    ("als_dataset_destroy", _i, [_vp]),
    ("als_dataset_counts", _i, [_vp, _pi64, _pi64, _pi64]),
    ("als_dataset_ids", _i, [_vp, _i, _pi64]),
    ("als_dataset_ratings", _i, [_vp, _pi32, _pi32, _pi16]),
    ("als_dataset_count_duplicates", _i, [_vp, _pi64]),
    ("als_dataset_shard_info", _i, [_vp, _i, _i, _i, _pi64, _pi64, _pi64, _pi64, _pi64]),
    ("als_dataset_set_slot_chunks", _i, [_vp, _i, _i]),
    ("als_dataset_slot_layout", _i, [_vp, _i, _i, _pi64, ctypes.POINTER(ctypes.c_int)]),
    ("als_dataset_shard_block", _i, [_vp, _i, _i, _i64, _pi64, _pi32, _pi16, _pi64]),
    ("als_dataset_shard_coo", _i, [_vp, _i, _i, _i64, _pi32, _pi32, _pi16]),
    ("als_dataset_slots", _i, [_vp, _i, _i, _pi64]),
    ("als_dataset_init_user_factors", _i, [_vp, _i, _u64, _i, _pf, _i64, _i64]),
    ("als_u01", _f, [_u64, _i64, ctypes.c_int32]),
    ("als_write_prediction_csv", _i, [ctypes.c_char_p, _pf, _i64, _i64, _pf, _i64, _i64, _i]),
    ("als_write_prediction_matrix_csv", _i, [ctypes.c_char_p, _pf, _i64, _i64]),
    ("als_feature_message_size", _i64, [_i64, _i]),
    ("als_feature_message_encode", _i, [ctypes.c_int32, _pi32, _i64, _pf, _i, _pu8, _i64, _pi64]),
    ("als_feature_message_decode", _i, [_pu8, _i64, _i, _pi32, _pi32, _i64, _pi64, _pf]),
    ("als_id_rating_encode", _i, [ctypes.c_int32, ctypes.c_int16, _pu8]),
    ("als_id_rating_decode", _i, [_pu8, _i64, _pi32, _pi16]),
    ("als_encode_feature_messages", _i, [_vp, _i, _i, _i, _pf, _i64, _pu8, _i64, _pi64, _pi64, _pi32, _pi64, _i64]),
]


def exported_symbols() -> list[str]:
    return [s[0] for s in SIGNATURES]


def lib():
    """Load libcfk_als.so (raises if it has not been built: run __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not found: the HIP extension is not built (python -c "
                              f"'import __graft_entry__; __graft_entry__.build()'); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status: int, fn: str) -> None:
    if status != ALS_OK:
        raise ALSError(status, fn, lib().als_last_error().decode(errors="replace"))


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)


def ptr(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))
