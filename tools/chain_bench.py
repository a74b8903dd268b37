"""Per-step latency of the fast sweep: one wave sweeps one cell (nb=1, G=1).

    python tools/chain_bench.py [k] [n]
cases: 'chain' = one item, n distinct users (the hot-item dependency chain);
       'runs'  = n ratings over n/64 items (runs of 64), distinct users;
       'wide'  = n ratings, G=64 groups (64 waves), to compare with one wave.
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "large-scale-recommendation_amd"))
import numpy as np

import mfhip
from mfhip import _lib as L

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
only = sys.argv[3] if len(sys.argv) > 3 else ""  # run only cases whose label starts with this


def run(u, i, groups, label, kern):
    if only and not label.startswith(only):
        return
    os.environ["MFHIP_TEST"] = f"fast_kernel={kern}"
    p = L.default_params()
    p.num_factors, p.num_blocks, p.mode, p.fast_waves, p.iterations = k, 1, L.MODE_FAST_F32, -groups, 1
    ctx = mfhip.Context(p)
    r = np.full(len(u), 3.0)
    ctx.prepare(u, i, r)
    ctx.run(1)
    ctx.sync()
    ctx.reset_stats()
    ctx.set_profiling(True)
    t0 = time.perf_counter()
    ctx.run(3)
    ctx.sync()
    t1 = time.perf_counter()
    st = ctx.stats()
    ns = st["kernel_ms"] * 1e6 / st["updates"]
    print(f"{label:28s} {kern:10s} k={k} n={len(u)} groups={groups} pads={st['pads']} kernel_ms/superstep="
          f"{st['kernel_ms']/3:.3f} ns/update(all waves)={ns:.1f} wall_ms={1e3*(t1-t0)/3:.3f}", flush=True)
    ctx.close()


users = np.arange(n, dtype=np.int32)
if os.environ.get("CHAIN_USERS"):  # a small user set cycled in order: rows stay cache-resident
    users = (users % int(os.environ["CHAIN_USERS"])).astype(np.int32)
for kern in ("substep",):
    run(users, np.zeros(n, np.int32), 1, "chain (1 item, 1 wave)", kern)
    run(users, (users // 64).astype(np.int32), 1, "runs of 64 (1 wave)", kern)
    rng = np.random.default_rng(0)
    run(users, rng.integers(0, 4096, n).astype(np.int32), 64, "random items, 64 groups", kern)
