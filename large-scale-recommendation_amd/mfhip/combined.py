"""Combined offline + online model.

Mirrors OnlineSpark.buildModelCombineOffline (sp/OnlineSpark.scala:26-162) on GPU-resident
factors: every micro-batch either
  * updates the model online -- one OfflineSpark.offlineDSGDUpdatesOnly sweep of the batch over
    num_partitions partitions (sp/OfflineSpark.scala:91-207, iterations = 1; MF_ONLINE_SPARK_SWEEP)
    -- and emits the touched user and item vectors (UpdateSeparatedHashMap.updates, :33-67), or,
  * every `offline_every`-th batch, refits from scratch on the whole rating history --
    OfflineSpark.offlineDSGD with empty initial factors and `iterations` sweeps (:68-89) -- and
    emits every vector.
The counters follow the reference (decrement, fire at <= 0, reset).  Every `checkpoint_every`-th
batch the model is written as an mf_save_model snapshot when `snapshot_dir` is given: the
localCheckpoint of the reference (:93-99) cuts RDD lineage; here it is a restartable file.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import numpy as np

from . import _lib as L
from .context import Context


class OnlineOfflineSpark:
    def __init__(self, num_factors: int, learning_rate: float = 0.01, num_partitions: int = 4,
                 offline_every: int = 10, checkpoint_every: int = 10, iterations: int = 10,
                 init: str = "pseudo_random", seed: int = 0, mode: str = "deterministic",
                 snapshot_dir: Optional[str] = None):
        self.k = num_factors
        self.P = num_partitions
        self.offline_every = offline_every
        self.checkpoint_every = checkpoint_every
        self.iterations = iterations
        self.snapshot_dir = snapshot_dir
        self._offline_cnt = offline_every
        self._checkpoint_cnt = checkpoint_every
        self._batches = 0
        p = L.default_params()
        p.num_factors = num_factors
        p.online_learning_rate = learning_rate
        p.online_init = L.INIT_SEEDED if init == "seeded" else L.INIT_PSEUDO_RANDOM
        p.seed = seed
        p.mode = L.MODE_FAST_F32 if mode == "fast" else L.MODE_DETERMINISTIC_F64
        self._params = p
        self.ctx = Context(p)
        self._hist = ([], [], [])  # ratings history (OnlineSpark.scala:71), as array chunks

    def close(self) -> None:
        self.ctx.close()

    def process(self, u, i, r) -> Tuple[Dict[int, np.ndarray], Dict[int, np.ndarray], bool]:
        """One micro-batch; returns (user updates, item updates, whether it was an offline refit)."""
        u = np.ascontiguousarray(u, np.int32)
        i = np.ascontiguousarray(i, np.int32)
        r = np.ascontiguousarray(r, np.float64)
        self._batches += 1
        self._checkpoint_cnt -= 1
        checkpoint = self._checkpoint_cnt <= 0
        if checkpoint:
            self._checkpoint_cnt = self.checkpoint_every
        self._offline_cnt -= 1
        offline = self._offline_cnt <= 0
        if offline:
            self._offline_cnt = self.offline_every
        for dst, src in zip(self._hist, (u, i, r)):
            dst.append(src)
        if not offline:
            self.ctx.online_update(u, i, r, L.ONLINE_SPARK_SWEEP, self.P)
            users, items = np.unique(u), np.unique(i)
        else:
            hu, hi, hr = (np.concatenate(x) for x in self._hist)
            fresh = Context(self._params)
            for _ in range(self.iterations):
                fresh.online_update(hu, hi, hr, L.ONLINE_SPARK_SWEEP, self.P)
            self.ctx.close()
            self.ctx = fresh
            users, items = np.unique(hu), np.unique(hi)
        uv, _ = self.ctx.lookup(L.SIDE_USER, users)
        iv, _ = self.ctx.lookup(L.SIDE_ITEM, items)
        if checkpoint and self.snapshot_dir:
            self.ctx.save(os.path.join(self.snapshot_dir, f"model_{self._batches:06d}.mfsnap"))
        return ({int(a): v for a, v in zip(users, uv)}, {int(a): v for a, v in zip(items, iv)}, offline)


class PSOfflineOnlineMF:
    """Parameter-server offline + online model (fl/mf/PSOfflineOnlineMF.scala:28-359) on GPU-resident
    factors, in its sequential serialisation (one worker, one PS shard, pull limits 1: every pull is
    answered before the next is sent, so the asynchronous protocol reduces to arrival order).

      * online (Online state, :139-149, :157-181): each rating is appended to the history `rs` and
        applied with SGDUpdater.delta -- user += delta_u on the worker, item += delta_i on the PS
        (:169-173, :250-252) -- i.e. MF_ONLINE_DELTA in arrival order;
      * batch trigger (:75-137): the PS drops every item vector (`params.clear()`, :287), the
        worker keeps its user vectors, then `iterations` passes over `rs` in insertion order (the
        `Random.shuffle(rs)` result is discarded, :113) re-pull items, which re-initialise from the
        FactorInitializer on first touch (:247-252), and push deltas (Batch state, :322-330).
        Ratings arriving during a batch are queued and applied online after it (:221-226), which
        is what calling `process` after `batch` does.
    Returned vectors are the model state after the call.  With emit_outputs=True every rating's
    worker output -- ps.output(user, userVec + deltaItemVec), userVec before the update (:176), the
    reference's stream out of this operator -- is kept in `self.output` after each call as (user
    ids, n x k vectors) in application order (mf_online_update_out; a batch keeps all its passes,
    iterations x n rows, as the reference emits them).  Off by default: per-rating records need
    the level-by-level replay instead of the one-launch online sweep, and n x k f64 per call."""

    def __init__(self, num_factors: int, learning_rate: float = 0.01, iterations: int = 10,
                 init: str = "pseudo_random", seed: int = 0, mode: str = "deterministic",
                 emit_outputs: bool = False):
        self.k = num_factors
        self.iterations = iterations
        self.emit_outputs = emit_outputs
        self.output = (np.empty(0, np.int32), np.empty((0, num_factors)))
        p = L.default_params()
        p.num_factors = num_factors
        p.online_learning_rate = learning_rate
        p.online_init = L.INIT_SEEDED if init == "seeded" else L.INIT_PSEUDO_RANDOM
        p.seed = seed
        p.mode = L.MODE_FAST_F32 if mode == "fast" else L.MODE_DETERMINISTIC_F64
        self._params = p
        self.ctx = Context(p)
        self._hist = ([], [], [])  # rs (:54)

    def close(self) -> None:
        self.ctx.close()

    def _vectors(self, users, items) -> Tuple[Dict[int, np.ndarray], Dict[int, np.ndarray]]:
        uv, _ = self.ctx.lookup(L.SIDE_USER, users)
        iv, _ = self.ctx.lookup(L.SIDE_ITEM, items)
        return {int(a): v for a, v in zip(users, uv)}, {int(a): v for a, v in zip(items, iv)}

    def process(self, u, i, r) -> Tuple[Dict[int, np.ndarray], Dict[int, np.ndarray]]:
        """Online ratings in arrival order; returns the touched user and item vectors."""
        u = np.ascontiguousarray(u, np.int32)
        i = np.ascontiguousarray(i, np.int32)
        r = np.ascontiguousarray(r, np.float64)
        for dst, src in zip(self._hist, (u, i, r)):
            dst.append(src)
        self._apply(self.ctx, [(u, i, r)])
        return self._vectors(np.unique(u), np.unique(i))

    def _apply(self, ctx: Context, passes) -> None:
        """SGDUpdater.delta updates in order (vectorUpdateAndPush, :167-180), keeping the outputs."""
        ids, outs = [], []
        for u, i, r in passes:
            if self.emit_outputs:
                uo, _ = ctx.online_update_out(u, i, r, L.ONLINE_DELTA, items=False)
                ids.append(u)
                outs.append(uo)
            else:
                ctx.online_update(u, i, r, L.ONLINE_DELTA)
        if self.emit_outputs:
            self.output = (np.concatenate(ids), np.concatenate(outs))

    def batch(self) -> Tuple[Dict[int, np.ndarray], Dict[int, np.ndarray]]:
        """Batch training over the whole history; returns every user and item vector."""
        if not self._hist[0]:
            return {}, {}
        hu, hi, hr = (np.concatenate(x) for x in self._hist)
        uids, uvecs = self.ctx.factors(L.SIDE_USER)
        fresh = Context(self._params)  # PS params.clear(): items re-initialise on first pull
        fresh.set_factors(L.SIDE_USER, uids, uvecs)  # worker userVectors survive the batch
        self._apply(fresh, [(hu, hi, hr)] * self.iterations)
        self.ctx.close()
        self.ctx = fresh
        return self._vectors(np.unique(hu), np.unique(hi))
