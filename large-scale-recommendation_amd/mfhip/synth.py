"""Seeded synthetic rating matrices with the shapes of BASELINE.json's configs.

Backed by lib/libmfsynth.so (csrc/synth.c): every value is a function of (seed, index), so
all ranks of a multi-GPU job generate identical data and the thread count does not matter.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
from dataclasses import dataclass

import numpy as np

from ._lib import PKG_DIR

SYNTH_PATH = os.path.join(os.path.dirname(PKG_DIR), "lib", "libmfsynth.so")

# name: (users, items, ratings, k, n_blocks)
CONFIGS = {
    "ML100K": (943, 1682, 100_000, 10, 4),
    "ML20M": (138_493, 26_744, 20_000_263, 64, 8),
    "NFLX": (480_189, 17_770, 100_480_507, 128, 8),
    "YAHOO": (1_823_179, 136_736, 717_872_016, 256, 8),
}

_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(SYNTH_PATH):
            raise ImportError(f"{SYNTH_PATH} missing; run __graft_entry__.build()")
        L = C.CDLL(SYNTH_PATH)
        L.mfs_generate.restype = C.c_int
        L.mfs_generate.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.c_uint64, C.c_uint64, C.c_uint64,
                                   C.c_double, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


@dataclass
class Ratings:
    u: np.ndarray
    i: np.ndarray
    r: np.ndarray
    test: np.ndarray

    def split(self):
        tr = ~self.test
        return (self.u[tr], self.i[tr], self.r[tr]), (self.u[self.test], self.i[self.test], self.r[self.test])


def generate(n_users: int, n_items: int, n: int, seed: int = 42, perm_seed: int = 1234, split_seed: int = 7,
             test_fraction: float = 0.1, threads: int | None = None) -> Ratings:
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        threads = max(1, min(threads, 32))
    u = np.empty(n, np.int32)
    i = np.empty(n, np.int32)
    r = np.empty(n, np.float64)
    t = np.empty(n, np.uint8)
    rc = _load().mfs_generate(n_users, n_items, n, seed, perm_seed, split_seed, test_fraction, threads,
                              u.ctypes.data, i.ctypes.data, r.ctypes.data, t.ctypes.data)
    if rc != 0:
        raise ValueError("bad synthetic shape")
    return Ratings(u, i, r, t.astype(bool))


def config(name: str, scale: float = 1.0, **kw) -> Ratings:
    nu, ni, n, _, _ = CONFIGS[name]
    return generate(max(1, int(nu * scale)), max(1, int(ni * scale)), max(1, int(n * scale)), **kw)


def fingerprint(*arrays) -> str:
    """sha256 over the raw bytes of the given arrays (pins a committed fixture to its data)."""
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).view(np.uint8).data)
    return h.hexdigest()
