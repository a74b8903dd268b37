"""Online MF on GPU micro-batches.

Replaces the per-rating operators of the reference's streaming jobs:
  * FlinkOnlineMF.buildModel (fl/mf/online/FlinkOnlineMF.scala:19-137): user operator +
    item operator with SGDUpdater.nextFactors; results equal the synchronous-feedback
    serialisation, i.e. ratings applied in arrival order with per-user FIFO
    (LockableStateWithQueue, fl/mf/utils/LockableState.scala:15-53).
  * OnlineSpark.buildModelWithMap (sp/OnlineSpark.scala:164-232): one
    OfflineSpark.offlineDSGDUpdatesOnly sweep per micro-batch (sp/OfflineSpark.scala:91-207).
  * The PS worker update (fl/mf/PSOfflineOnlineMF.scala:167-180): SGDUpdater.delta + "vec + delta".
A batch is ONE persistent launch (k_online_sweep): the updates of an item run in sequence order
on one wave (the item row stays in registers), and an update whose user was updated earlier in
the batch waits for that user's ticket, so the GPU result is the sequential result; the wave
lists and tickets are built on the device (kernels_online.hip).  Per-rating output records
(Context.online_update_out) use the level-by-level replay instead (one launch per dependency
level: no two updates of a level share a row).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .context import Context
from .core import FactorVector, Rating, SGDUpdater


class OnlineMF:
    """A GPU-resident online model.  flavour: "flink" (arrival order), "spark" (Spark sweep order
    over num_partitions), "ps" (delta path).  init: "pseudo_random" (new Random(id)) or "seeded"."""

    FLAVOURS = {"flink": L.ONLINE_NEXT_FACTORS, "ps": L.ONLINE_DELTA, "spark": L.ONLINE_SPARK_SWEEP}

    def __init__(self, num_factors: int, learning_rate: float = 0.01, flavour: str = "flink",
                 num_partitions: int = 4, init: str = "pseudo_random", seed: int = 0, mode: str = "deterministic",
                 context: Optional[Context] = None):
        self.flavour = flavour
        self.num_partitions = num_partitions
        if context is None:
            p = L.default_params()
            p.num_factors = num_factors
            p.online_learning_rate = learning_rate
            p.online_init = L.INIT_SEEDED if init == "seeded" else L.INIT_PSEUDO_RANDOM
            p.seed = seed
            p.mode = L.MODE_FAST_F32 if mode == "fast" else L.MODE_DETERMINISTIC_F64
            context = Context(p)
        self.ctx = context
        self.k = num_factors

    @staticmethod
    def from_updater(updater: SGDUpdater, num_factors: int, **kw) -> "OnlineMF":
        return OnlineMF(num_factors, learning_rate=updater.learningRate, **kw)

    def update(self, batch) -> Tuple[int, int]:
        """Apply one micro-batch; returns (touched users, touched items)."""
        if isinstance(batch, tuple) and len(batch) == 3 and not np.isscalar(batch[0]):
            u, i, r = batch
        else:
            b = [x if isinstance(x, tuple) else (x.user, x.item, x.rating) for x in batch]
            u = [x[0] for x in b]
            i = [x[1] for x in b]
            r = [x[2] for x in b]
        return self.ctx.online_update(u, i, r, self.FLAVOURS[self.flavour], self.num_partitions)

    def vectors(self, side: int, ids) -> Tuple[np.ndarray, np.ndarray]:
        return self.ctx.lookup(side, ids)

    def user_vectors(self) -> List[FactorVector]:
        ids, vecs = self.ctx.factors(L.SIDE_USER)
        return [FactorVector(int(a), v) for a, v in zip(ids, vecs)]

    def item_vectors(self) -> List[FactorVector]:
        ids, vecs = self.ctx.factors(L.SIDE_ITEM)
        return [FactorVector(int(a), v) for a, v in zip(ids, vecs)]
