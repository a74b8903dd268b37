"""oracle/coracle.py -- TEST INFRASTRUCTURE ONLY: ctypes view of oracle/build/libmforacle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libmforacle.so")

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_jr_next_int.argtypes = [C.c_int64, C.c_int32, _i32p]
        L.orc_jr_next_int_bound.argtypes = [C.c_int64, C.c_int32, C.c_int32, _i32p]
        L.orc_jr_next_double.argtypes = [C.c_int64, C.c_int32, _f64p]
        L.orc_scala_shuffle.argtypes = [C.c_int64, C.c_int64, _i32p]
        L.orc_block_of.argtypes = [C.c_int32, C.c_int64, C.c_int32]
        L.orc_block_of.restype = C.c_int32
        L.orc_random_factors.argtypes = [C.c_int64, C.c_int32, _f64p]
        L.orc_learning_rate.argtypes = [C.c_int, C.c_double, C.c_int32, C.c_double, C.c_double]
        L.orc_learning_rate.restype = C.c_double
        L.orc_dsgd_fit.argtypes = [C.c_int32, C.c_int32, C.c_double, C.c_double, C.c_int32,
                                   C.c_double, C.c_int32, C.c_int64, C.c_int32, C.c_int64,
                                   _i32p, _i32p, _f64p, C.c_int64,
                                   C.POINTER(C.c_double), C.POINTER(C.c_int64)]
        L.orc_dsgd_fit.restype = C.c_void_p
        L.orc_model_count.argtypes = [C.c_void_p, C.c_int32]
        L.orc_model_count.restype = C.c_int64
        L.orc_model_get.argtypes = [C.c_void_p, C.c_int32, _i32p, _f64p]
        L.orc_model_predict.argtypes = [C.c_void_p, _i32p, _i32p, C.c_int64, _f64p, _u8p]
        L.orc_model_free.argtypes = [C.c_void_p]
        L.orc_block_update.argtypes = [_f64p, _i32p, _i32p, C.c_int64, _f64p, _i32p, _f64p, _i32p,
                                       C.c_int32, C.c_int32, C.c_int32, C.c_int64, C.c_double,
                                       C.c_int32, C.c_double, C.c_double]
        L.orc_online_apply.argtypes = [_i32p, _i32p, _f64p, C.c_int64, _f64p, _f64p, C.c_int32,
                                       C.c_double]
        L.orc_dsgd_apply.argtypes = [_i32p, _i32p, _f64p, C.c_int64, _f64p, _f64p, _f64p, _f64p, C.c_int32,
                                     C.c_double]
        _lib = L
    return _lib


def next_int(seed: int, count: int) -> np.ndarray:
    out = np.empty(count, np.int32)
    lib().orc_jr_next_int(seed, count, out)
    return out


def next_int_bound(seed: int, bound: int, count: int) -> np.ndarray:
    out = np.empty(count, np.int32)
    lib().orc_jr_next_int_bound(seed, bound, count, out)
    return out


def next_double(seed: int, count: int) -> np.ndarray:
    out = np.empty(count, np.float64)
    lib().orc_jr_next_double(seed, count, out)
    return out


def scala_shuffle(seed: int, n: int) -> np.ndarray:
    out = np.empty(max(n, 1), np.int32)
    lib().orc_scala_shuffle(seed, n, out)
    return out[:n]


def block_of(id_: int, seed: int, n_blocks: int) -> int:
    return int(lib().orc_block_of(id_, seed, n_blocks))


def learning_rate(method: int, lr: float, iteration: int, lam: float, arg: float = 0.0) -> float:
    return float(lib().orc_learning_rate(method, lr, iteration, lam, arg))


class Model:
    """Result of orc_dsgd_fit: factors keyed by id (ascending), plus sweep timing."""

    def __init__(self, handle, k: int, sweep_seconds: float, updates: int):
        self.h = handle
        self.k = k
        self.sweep_seconds = sweep_seconds
        self.updates = updates

    def factors(self, side: int):
        L = lib()
        n = L.orc_model_count(self.h, side)
        ids = np.empty(max(n, 1), np.int32)
        vecs = np.empty((max(n, 1), self.k), np.float64)
        L.orc_model_get(self.h, side, ids, vecs)
        return ids[:n], vecs[:n]

    def predict(self, u: np.ndarray, i: np.ndarray):
        n = len(u)
        out = np.empty(max(n, 1), np.float64)
        found = np.empty(max(n, 1), np.uint8)
        lib().orc_model_predict(self.h, np.ascontiguousarray(u, np.int32),
                                np.ascontiguousarray(i, np.int32), n, out, found)
        return out[:n], found[:n].astype(bool)

    def rmse(self, u, i, r) -> tuple[float, int]:
        pred, found = self.predict(u, i)
        d = (np.asarray(r, np.float64) - pred)[found]
        return (float(np.sqrt(np.mean(d * d))) if len(d) else float("nan")), int(found.sum())

    def close(self):
        if self.h:
            lib().orc_model_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def dsgd_fit(u, i, r, k=10, iterations=10, lam=1.0, lr=0.001, lr_method=0, lr_arg=0.0,
             n_blocks=1, seed=0, threads=1, max_supersteps=-1) -> Model:
    u = np.ascontiguousarray(u, np.int32)
    i = np.ascontiguousarray(i, np.int32)
    r = np.ascontiguousarray(r, np.float64)
    secs = C.c_double(0.0)
    ups = C.c_int64(0)
    h = lib().orc_dsgd_fit(k, iterations, lam, lr, lr_method, lr_arg, n_blocks, seed, threads,
                           max_supersteps, u, i, r, len(u), C.byref(secs), C.byref(ups))
    return Model(h, k, secs.value, ups.value)


def block_update(r, uidx, iidx, users, uomega, items, iomega, k, iteration, rating_block_id, seed,
                 lr, lr_method, lr_arg, lam):
    """orc_block_update on copies; returns (users, items)."""
    users = np.ascontiguousarray(users, np.float64).copy()
    items = np.ascontiguousarray(items, np.float64).copy()
    lib().orc_block_update(np.ascontiguousarray(r, np.float64), np.ascontiguousarray(uidx, np.int32),
                           np.ascontiguousarray(iidx, np.int32), len(r), users,
                           np.ascontiguousarray(uomega, np.int32), items,
                           np.ascontiguousarray(iomega, np.int32), k, iteration, rating_block_id,
                           seed, lr, lr_method, lr_arg, lam)
    return users, items


def online_apply(urow, irow, r, users, items, k, lr):
    """orc_online_apply: sequential SGDUpdater.nextFactors over row indices, in place."""
    lib().orc_online_apply(np.ascontiguousarray(urow, np.int32), np.ascontiguousarray(irow, np.int32),
                           np.ascontiguousarray(r, np.float64), len(r), users, items, k, lr)


def dsgd_apply(urow, irow, r, users, items, reg_u, reg_i, k, eta):
    """orc_dsgd_apply: sequential regularised DSGD updates in the given order, in place."""
    lib().orc_dsgd_apply(np.ascontiguousarray(urow, np.int32), np.ascontiguousarray(irow, np.int32),
                         np.ascontiguousarray(r, np.float64), len(r), users, items,
                         np.ascontiguousarray(reg_u, np.float64), np.ascontiguousarray(reg_i, np.float64), k, eta)
