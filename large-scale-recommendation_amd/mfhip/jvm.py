"""JVM-compatible RNG helpers exported by libmfhip (no GPU needed)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def shuffle(seed: int, n: int) -> np.ndarray:
    """scala.util.Random(seed).shuffle(0 until n)."""
    out = np.empty(max(n, 1), np.int32)
    L.check(L.lib().mf_jvm_shuffle(int(seed), int(n), L.ptr(out, C.c_int32)))
    return out[:n]


def block_of(id_: int, seed: int, n_blocks: int) -> int:
    """new Random(id ^ seed).nextInt(numBlocks) (DSGDforMF.scala:531-533)."""
    v = C.c_int32(0)
    L.check(L.lib().mf_jvm_block_of(int(id_), int(seed), int(n_blocks), C.byref(v)))
    return v.value


def random_factors(rng_seed: int, k: int) -> np.ndarray:
    """k x new Random(rng_seed).nextDouble()."""
    out = np.empty(max(k, 1), np.float64)
    L.check(L.lib().mf_jvm_random_factors(int(rng_seed), int(k), L.ptr(out, C.c_double)))
    return out[:k]


def learning_rate(method: int, lr: float, iteration: int, lam: float, arg: float = 0.0) -> float:
    v = C.c_double(0.0)
    L.check(L.lib().mf_learning_rate(int(method), float(lr), int(iteration), float(lam), float(arg), C.byref(v)))
    return v.value
