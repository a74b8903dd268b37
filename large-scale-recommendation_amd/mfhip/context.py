"""Thin object wrapper of an mf_ctx (one model on one or more GPUs)."""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from ._lib import as_f64, as_i32, check, ptr, same_length


class Context:
    """Owns an mf_ctx.  mode: "deterministic" (bit-exact f64 replay) or "fast" (f32)."""

    def __init__(self, params: L.mf_params, devices: Optional[Sequence[int]] = None, n_devices: int = 1,
                 rank: Optional[Tuple[int, int, int, bytes]] = None):
        self.params = params
        self.k = int(params.num_factors)
        self._h = C.c_void_p(None)
        lib = L.lib()
        if rank is not None:  # (device, nranks, rank, uid)
            dev, nranks, r, uid = rank
            ub = (C.c_uint8 * L.UID_BYTES).from_buffer_copy(uid.ljust(L.UID_BYTES, b"\0"))
            check(lib.mf_create_rank(C.byref(params), dev, nranks, r, ub, C.byref(self._h)))
        else:
            if devices is not None:
                arr = (C.c_int * len(devices))(*devices)
                check(lib.mf_create(C.byref(params), arr, len(devices), C.byref(self._h)))
            else:
                check(lib.mf_create(C.byref(params), None, n_devices, C.byref(self._h)))

    # -- lifecycle -------------------------------------------------------------
    def close(self) -> None:
        if self._h and self._h.value:
            check(L.lib().mf_destroy(self._h))
            self._h = C.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * L.UID_BYTES)()
        check(L.lib().mf_comm_unique_id(buf))
        return bytes(buf)

    # -- DSGD ------------------------------------------------------------------
    def fit(self, u, i, r) -> None:
        u, i, r = as_i32(u), as_i32(i), as_f64(r)
        same_length(u, i, r)
        check(L.lib().mf_dsgd_fit(self._h, ptr(u, C.c_int32), ptr(i, C.c_int32), ptr(r, C.c_double), len(u)))

    def prepare(self, u, i, r) -> None:
        u, i, r = as_i32(u), as_i32(i), as_f64(r)
        same_length(u, i, r)
        check(L.lib().mf_dsgd_prepare(self._h, ptr(u, C.c_int32), ptr(i, C.c_int32), ptr(r, C.c_double), len(u)))

    def run(self, supersteps: int) -> None:
        check(L.lib().mf_dsgd_run(self._h, int(supersteps)))

    def sync(self) -> None:
        check(L.lib().mf_sync(self._h))

    def restart(self) -> None:
        """Factors back to their initial values and superstep 0; blocking and schedule kept."""
        check(L.lib().mf_dsgd_restart(self._h))

    @property
    def superstep(self) -> int:
        v = C.c_int64(0)
        check(L.lib().mf_dsgd_superstep(self._h, C.byref(v)))
        return v.value

    @superstep.setter
    def superstep(self, done: int) -> None:
        check(L.lib().mf_dsgd_set_superstep(self._h, int(done)))

    # -- factors ---------------------------------------------------------------
    def num_factors(self, side: int) -> int:
        v = C.c_int64(0)
        check(L.lib().mf_num_factors(self._h, side, C.byref(v)))
        return v.value

    def factors(self, side: int) -> Tuple[np.ndarray, np.ndarray]:
        n = self.num_factors(side)
        ids = np.empty(max(n, 1), np.int32)
        vecs = np.empty((max(n, 1), self.k), np.float64)
        w = C.c_int64(0)
        check(L.lib().mf_get_factors(self._h, side, ptr(ids, C.c_int32), ptr(vecs, C.c_double), n, C.byref(w)))
        return ids[:w.value], vecs[:w.value]

    def set_factors(self, side: int, ids, vecs) -> None:
        ids = as_i32(ids)
        vecs = as_f64(vecs)
        if vecs.size != len(ids) * self.k:
            raise ValueError(f"vecs must hold len(ids) x k = {len(ids)} x {self.k} values, got {vecs.size}")
        vecs = vecs.reshape(len(ids), self.k)
        check(L.lib().mf_set_factors(self._h, side, ptr(ids, C.c_int32), ptr(vecs, C.c_double), len(ids)))

    def lookup(self, side: int, ids) -> Tuple[np.ndarray, np.ndarray]:
        ids = as_i32(ids)
        n = len(ids)
        out = np.empty((max(n, 1), self.k), np.float64)
        found = np.empty(max(n, 1), np.uint8)
        check(L.lib().mf_lookup(self._h, side, ptr(ids, C.c_int32), n, ptr(out, C.c_double), ptr(found, C.c_uint8)))
        return out[:n], found[:n].astype(bool)

    # -- evaluation ------------------------------------------------------------
    def predict(self, u, i) -> Tuple[np.ndarray, np.ndarray]:
        u, i = as_i32(u), as_i32(i)
        n = same_length(u, i)
        out = np.empty(max(n, 1), np.float64)
        found = np.empty(max(n, 1), np.uint8)
        check(L.lib().mf_predict(self._h, ptr(u, C.c_int32), ptr(i, C.c_int32), n, ptr(out, C.c_double),
                                 ptr(found, C.c_uint8)))
        return out[:n], found[:n].astype(bool)

    def rmse(self, u, i, r) -> Tuple[float, int]:
        u, i, r = as_i32(u), as_i32(i), as_f64(r)
        same_length(u, i, r)
        v = C.c_double(0.0)
        m = C.c_int64(0)
        check(L.lib().mf_rmse(self._h, ptr(u, C.c_int32), ptr(i, C.c_int32), ptr(r, C.c_double), len(u),
                              C.byref(v), C.byref(m)))
        return v.value, m.value

    def empirical_risk(self, u, i, r, lam: float) -> float:
        u, i, r = as_i32(u), as_i32(i), as_f64(r)
        same_length(u, i, r)
        v = C.c_double(0.0)
        check(L.lib().mf_empirical_risk(self._h, ptr(u, C.c_int32), ptr(i, C.c_int32), ptr(r, C.c_double), len(u),
                                        float(lam), C.byref(v)))
        return v.value

    # -- online ----------------------------------------------------------------
    def online_update(self, u, i, r, flavour: int = L.ONLINE_NEXT_FACTORS, num_partitions: int = 0):
        u, i, r = as_i32(u), as_i32(i), as_f64(r)
        same_length(u, i, r)
        tu, ti = C.c_int64(0), C.c_int64(0)
        check(L.lib().mf_online_update(self._h, ptr(u, C.c_int32), ptr(i, C.c_int32), ptr(r, C.c_double), len(u),
                                       flavour, num_partitions, C.byref(tu), C.byref(ti)))
        return tu.value, ti.value

    def online_update_out(self, u, i, r, flavour: int = L.ONLINE_NEXT_FACTORS, items: bool = True):
        """online_update plus the per-rating records the operators emit (mf_online_update_out):
        NEXT_FACTORS -> (user', item') per rating (FlinkOnlineMF.scala:131-135); DELTA ->
        (userVec + deltaItemVec, deltaItemVec) per rating (PSOfflineOnlineMF.scala:174-176).
        items=False: the item records are not produced (None; no n x k buffer, no copy back).
        Per-rating records need the level-by-level replay, slower than online_update's sweep."""
        u, i, r = as_i32(u), as_i32(i), as_f64(r)
        n = same_length(u, i, r)
        uo = np.empty((max(n, 1), self.k), np.float64)
        io = np.empty((max(n, 1), self.k), np.float64) if items else None
        tu, ti = C.c_int64(0), C.c_int64(0)
        check(L.lib().mf_online_update_out(self._h, ptr(u, C.c_int32), ptr(i, C.c_int32), ptr(r, C.c_double), n,
                                           flavour, 0, C.byref(tu), C.byref(ti), ptr(uo, C.c_double),
                                           ptr(io, C.c_double) if items else None))
        return uo[:n], (io[:n] if items else None)

    # -- snapshots (TemporaryPath persistence, DSGDforMF.scala:291-296, 330-349) --
    def save(self, path: str) -> None:
        check(L.lib().mf_save_model(self._h, path.encode()))

    def load(self, path: str) -> int:
        """Set both factor sides from a snapshot; returns the stored superstep counter (to resume
        a fit: prepare(same ratings), load(path), set_superstep(counter), run(...))."""
        step = C.c_int64(0)
        check(L.lib().mf_load_model(self._h, path.encode(), C.byref(step)))
        return step.value

    # -- stats -----------------------------------------------------------------
    def set_profiling(self, on: bool) -> None:
        check(L.lib().mf_set_profiling(self._h, 1 if on else 0))

    def stats(self) -> dict:
        s = L.mf_stats()
        check(L.lib().mf_get_stats(self._h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in L.mf_stats._fields_ if not f.startswith("reserved")}

    def plan_digest(self) -> tuple:
        """(FNV digest of the device schedule, pair records) after prepare (mf_debug_plan_digest)."""
        out = (C.c_uint64 * 2)()
        check(L.lib().mf_debug_plan_digest(self._h, out))
        return int(out[0]), int(out[1])

    def reset_stats(self) -> None:
        check(L.lib().mf_reset_stats(self._h))


def block_update(r, uidx, iidx, users, uomega, items, iomega, k, iteration, rating_block_id, seed, lr,
                 lr_method=0, lr_arg=0.0, lam=1.0, ctx: Optional[Context] = None):
    """mf_block_update: exact updateLocalFactors (DSGDforMF.scala:378-418) on copies of users/items."""
    own = ctx is None
    if own:
        p = L.default_params()
        p.num_factors = k
        ctx = Context(p)
    try:
        r, uidx, iidx = as_f64(r), as_i32(uidx), as_i32(iidx)
        same_length(r, uidx, iidx)
        users = as_f64(users).copy()
        items = as_f64(items).copy()
        uomega, iomega = as_i32(uomega), as_i32(iomega)
        check(L.lib().mf_block_update(ctx._h, ptr(r, C.c_double), ptr(uidx, C.c_int32), ptr(iidx, C.c_int32), len(r),
                                      ptr(users, C.c_double), ptr(uomega, C.c_int32), users.shape[0],
                                      ptr(items, C.c_double), ptr(iomega, C.c_int32), items.shape[0], k, iteration,
                                      rating_block_id, seed, lr, lr_method, lr_arg, lam))
        return users, items
    finally:
        if own:
            ctx.close()
