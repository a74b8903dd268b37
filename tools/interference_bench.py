"""Hot-chain slowdown under background load: one hot item with H ratings (its own group) plus
B background ratings on other items, G groups, one rating block.  Superstep time ~ hot wave."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "large-scale-recommendation_amd"))
import numpy as np

import mfhip
from mfhip import _lib as L

k = 128


def run(H, B, groups, kern, nb=1):
    os.environ["MFHIP_TEST"] = f"fast_kernel={kern}"
    rng = np.random.default_rng(1)
    nu = max(H, B // 4 + 1)
    u = np.concatenate([rng.permutation(nu)[:H], rng.integers(0, nu, B)]).astype(np.int32)
    i = np.concatenate([np.zeros(H, np.int32), rng.integers(1, 8192, B).astype(np.int32)])
    p = L.default_params()
    p.num_factors, p.num_blocks, p.mode, p.fast_waves, p.iterations = k, nb, L.MODE_FAST_F32, -groups, 1
    ctx = mfhip.Context(p)
    ctx.prepare(u, i, np.full(len(u), 3.0))
    ctx.run(nb)
    ctx.sync()
    ctx.reset_stats()
    ctx.set_profiling(True)
    ctx.run(3 * nb)
    ctx.sync()
    st = ctx.stats()
    per_ss = st["kernel_ms"] / (3 * nb)
    print(f"{kern:10s} H={H:7d} B={B:9d} G={groups:4d} nb={nb} superstep_ms={per_ss:8.3f} "
          f"hot_ns/step={per_ss*1e6/max(H//nb,1):8.1f} agg_Mups={st['updates']/(st['kernel_ms']/1e3)/1e6:8.1f}", flush=True)
    ctx.close()


for kern in ("substep",):
    run(20000, 0, 64, kern)
    run(20000, 200000, 64, kern)
    run(20000, 2000000, 64, kern)
    run(20000, 2000000, 256, kern)
    run(20000, 8000000, 256, kern)
