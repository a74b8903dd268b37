"""ctypes binding of libmfhip.so (include/mfhip.h; test hooks: include/mfhip_testing.h).

This is the Python-side equivalent of the JNI shim in INTEGRATION.md: plain pointers and
sizes, status codes mapped to exceptions.  The library has no CPU fallback; loading fails
loudly when the shared object is missing, and context creation fails with MFNoDeviceError
when no GPU is visible.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MFHIP_LIB", os.path.join(os.path.dirname(PKG_DIR), "lib", "libmfhip.so"))

MF_OK = 0
MF_ERR_INVALID = -1
MF_ERR_HIP = -2
MF_ERR_NOT_FITTED = -3
MF_ERR_NO_DEVICE = -4
MF_ERR_COMM = -5
MF_ERR_CAPACITY = -6
MF_ERR_STATE = -7

MODE_DETERMINISTIC_F64 = 0
MODE_FAST_F32 = 1
BLOCKING_REFERENCE = 0
BLOCKING_BALANCED = 1
SIDE_USER = 0
SIDE_ITEM = 1
ONLINE_NEXT_FACTORS = 0
ONLINE_DELTA = 1
ONLINE_SPARK_SWEEP = 2
INIT_PSEUDO_RANDOM = 0
INIT_SEEDED = 1
UID_BYTES = 128


class MFError(RuntimeError):
    """Non-zero status from libmfhip (the JNI shim raises RuntimeException, like the reference)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[mfhip {code}] {msg}")
        self.code = code


class MFNoDeviceError(MFError):
    pass


class mf_params(C.Structure):
    _fields_ = [
        ("num_factors", C.c_int32),
        ("iterations", C.c_int32),
        ("lambda_", C.c_double),
        ("learning_rate", C.c_double),
        ("lr_method", C.c_int32),
        ("lr_arg", C.c_double),
        ("num_blocks", C.c_int32),
        ("seed", C.c_int64),
        ("has_seed", C.c_int32),
        ("mode", C.c_int32),
        ("online_learning_rate", C.c_double),
        ("online_init", C.c_int32),
        ("fast_waves", C.c_int32),
        ("fast_blocking", C.c_int32),
        ("reserved", C.c_int32 * 6),
    ]


class mf_stats(C.Structure):
    _fields_ = [
        ("updates", C.c_int64),
        ("supersteps", C.c_int64),
        ("kernel_launches", C.c_int64),
        ("kernel_ms", C.c_double),
        ("algorithmic_bytes", C.c_double),
        ("levels", C.c_int64),
        ("groups", C.c_int32),
        ("reserved0", C.c_int32),
        ("pads", C.c_int64),
        ("moved_bytes", C.c_double),
    ]


# Every symbol include/mfhip.h declares (tests check the library exports all of them).
EXPORTS = [
    "mf_params_init", "mf_last_error", "mf_version", "mf_device_count", "mf_create",
    "mf_comm_unique_id", "mf_create_rank", "mf_destroy", "mf_dsgd_fit", "mf_dsgd_prepare",
    "mf_dsgd_run", "mf_dsgd_superstep", "mf_dsgd_set_superstep", "mf_sync", "mf_num_factors",
    "mf_get_factors", "mf_set_factors", "mf_predict", "mf_rmse", "mf_empirical_risk",
    "mf_block_update", "mf_online_update", "mf_lookup", "mf_set_profiling", "mf_get_stats",
    "mf_reset_stats", "mf_jvm_shuffle", "mf_jvm_block_of", "mf_jvm_random_factors",
    "mf_learning_rate", "mf_get_params", "mf_read_ratings", "mf_save_model", "mf_load_model",
    "mf_dsgd_restart", "mf_online_update_out",
]
# The test hooks include/mfhip_testing.h declares (not product surface; same library).
TESTING_EXPORTS = [
    "mf_debug_levels", "mf_debug_fast_schedule", "mf_debug_fast_split", "mf_debug_ring_schedule",
    "mf_debug_plan_digest", "mf_fast_plan_window", "mf_fast_kernel_name", "mf_debug_build_flags",
    "mf_debug_device_bytes",
]

_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_f64p = C.POINTER(C.c_double)
_u8p = C.POINTER(C.c_uint8)
_ctxp = C.c_void_p

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libmfhip.so not found at {LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP path has no fallback)")
    L = C.CDLL(LIB_PATH)
    sig = {
        "mf_params_init": (None, [C.POINTER(mf_params)]),
        "mf_last_error": (C.c_char_p, []),
        "mf_version": (C.c_char_p, []),
        "mf_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "mf_create": (C.c_int, [C.POINTER(mf_params), C.POINTER(C.c_int), C.c_int, C.POINTER(_ctxp)]),
        "mf_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
        "mf_create_rank": (C.c_int, [C.POINTER(mf_params), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8),
                                     C.POINTER(_ctxp)]),
        "mf_destroy": (C.c_int, [_ctxp]),
        "mf_dsgd_fit": (C.c_int, [_ctxp, _i32p, _i32p, _f64p, C.c_int64]),
        "mf_dsgd_prepare": (C.c_int, [_ctxp, _i32p, _i32p, _f64p, C.c_int64]),
        "mf_dsgd_run": (C.c_int, [_ctxp, C.c_int64]),
        "mf_dsgd_superstep": (C.c_int, [_ctxp, _i64p]),
        "mf_dsgd_set_superstep": (C.c_int, [_ctxp, C.c_int64]),
        "mf_sync": (C.c_int, [_ctxp]),
        "mf_num_factors": (C.c_int, [_ctxp, C.c_int, _i64p]),
        "mf_get_factors": (C.c_int, [_ctxp, C.c_int, _i32p, _f64p, C.c_int64, _i64p]),
        "mf_set_factors": (C.c_int, [_ctxp, C.c_int, _i32p, _f64p, C.c_int64]),
        "mf_predict": (C.c_int, [_ctxp, _i32p, _i32p, C.c_int64, _f64p, _u8p]),
        "mf_rmse": (C.c_int, [_ctxp, _i32p, _i32p, _f64p, C.c_int64, _f64p, _i64p]),
        "mf_empirical_risk": (C.c_int, [_ctxp, _i32p, _i32p, _f64p, C.c_int64, C.c_double, _f64p]),
        "mf_block_update": (C.c_int, [_ctxp, _f64p, _i32p, _i32p, C.c_int64, _f64p, _i32p, C.c_int64, _f64p,
                                      _i32p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_double,
                                      C.c_int, C.c_double, C.c_double]),
        "mf_online_update": (C.c_int, [_ctxp, _i32p, _i32p, _f64p, C.c_int64, C.c_int, C.c_int, _i64p, _i64p]),
        "mf_lookup": (C.c_int, [_ctxp, C.c_int, _i32p, C.c_int64, _f64p, _u8p]),
        "mf_set_profiling": (C.c_int, [_ctxp, C.c_int]),
        "mf_get_stats": (C.c_int, [_ctxp, C.POINTER(mf_stats)]),
        "mf_reset_stats": (C.c_int, [_ctxp]),
        "mf_jvm_shuffle": (C.c_int, [C.c_int64, C.c_int64, _i32p]),
        "mf_jvm_block_of": (C.c_int, [C.c_int32, C.c_int64, C.c_int32, _i32p]),
        "mf_jvm_random_factors": (C.c_int, [C.c_int64, C.c_int32, _f64p]),
        "mf_learning_rate": (C.c_int, [C.c_int, C.c_double, C.c_int32, C.c_double, C.c_double, _f64p]),
        "mf_debug_levels": (C.c_int, [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), _i32p, C.c_int64, _i32p]),
        "mf_debug_fast_schedule": (C.c_int, [_i32p, _i32p, C.c_int64, C.c_int32, C.c_int64, C.c_int32, C.c_int32,
                                             C.c_int32, C.c_int32, _i32p, _i32p, _i32p, _i64p]),
        "mf_debug_fast_split": (C.c_int, [_i32p, _i32p, C.c_int64, C.c_int32, C.c_int64, C.c_int32, C.c_int32,
                                          C.c_int32, C.c_int32, C.c_int32, _i32p, _i32p, _i32p, _i64p, _i32p]),
        "mf_fast_plan_window": (C.c_int, [C.c_int32, _i32p]),
        "mf_fast_kernel_name": (C.c_char_p, [C.c_int32]),
        "mf_get_params": (C.c_int, [C.c_void_p, C.POINTER(mf_params)]),
        "mf_read_ratings": (C.c_int, [C.c_char_p, C.c_char, C.c_int32, _i32p, _i32p, _f64p, C.c_int64, _i64p]),
        "mf_save_model": (C.c_int, [C.c_void_p, C.c_char_p]),
        "mf_load_model": (C.c_int, [C.c_void_p, C.c_char_p, _i64p]),
        "mf_dsgd_restart": (C.c_int, [_ctxp]),
        "mf_online_update_out": (C.c_int, [_ctxp, _i32p, _i32p, _f64p, C.c_int64, C.c_int, C.c_int, _i64p, _i64p,
                                           _f64p, _f64p]),
        "mf_debug_ring_schedule": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int64, _i32p, _i32p, _i32p, _i32p]),
        "mf_debug_plan_digest": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
        "mf_debug_build_flags": (C.c_int32, []),
        "mf_debug_device_bytes": (C.c_int, [_i64p]),
    }
    for name, (res, args) in sig.items():
        if name in TESTING_EXPORTS and not hasattr(L, name):
            continue  # an older build (A/B runs): its test hooks may predate this binding
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status: int) -> None:
    if status != MF_OK:
        msg = lib().mf_last_error().decode(errors="replace")
        if status == MF_ERR_NO_DEVICE:
            raise MFNoDeviceError(status, msg)
        raise MFError(status, msg)


def ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def as_i32(a) -> np.ndarray:
    """Ids as the reference's Int: values outside int32 are rejected, not wrapped."""
    arr = np.asarray(a)
    if arr.dtype != np.int32 and arr.size:
        if arr.dtype.kind not in "iub":
            raise ValueError(f"ids must be integers, got {arr.dtype}")
        lo, hi = int(arr.min()), int(arr.max())
        if lo < -2**31 or hi >= 2**31:
            raise ValueError(f"id out of the Int range: [{lo}, {hi}]")
    return np.ascontiguousarray(arr, dtype=np.int32)


def same_length(*arrays) -> int:
    """Rating columns must be parallel arrays: the C side reads len(first) elements of each."""
    n = len(arrays[0])
    for a in arrays[1:]:
        if len(a) != n:
            raise ValueError(f"columns differ in length: {[len(x) for x in arrays]}")
    return n


def as_f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def default_params() -> mf_params:
    p = mf_params()
    lib().mf_params_init(C.byref(p))
    return p


def device_count() -> int:
    n = C.c_int(0)
    check(lib().mf_device_count(C.byref(n)))
    return n.value


def version() -> str:
    return lib().mf_version().decode()
