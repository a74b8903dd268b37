#!/usr/bin/env python3
"""Online MF on top of an offline DSGD model (BASELINE.json config 5, SURVEY.md 8d ONLINE).

    python tools/online_bench.py [--config NFLX] [--epochs 2] [--batches 10] [--batch 1000000]
                                 [--flavour flink|ps|spark] [--mode fast|det] [--out file.json]

Fits the config's training split with fast DSGD for --epochs epochs, then streams --batches
micro-batches of --batch ratings drawn from the same generator (other seed: new ratings of the
same users and items, plus whatever unseen ids the draw produces) through mf_online_update
(SGDUpdater.nextFactors in arrival order, core/FactorUpdater.scala:35-54; FlinkOnlineMF
per-user FIFO).  Reports ratings/s per batch (host planning + H2D + kernels, end to end) next to
the 10M ratings/s target of 100-ms micro-batches.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-recommendation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="NFLX")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--batches", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--flavour", default="flink", choices=["flink", "ps", "spark"])
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--mode", default="fast", choices=["fast", "det"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import numpy as np
    import mfhip
    from mfhip import _lib as L
    from mfhip import synth

    nu, ni, nr, k, nb = synth.CONFIGS[a.config]
    nu, ni, nr = max(1, int(nu * a.scale)), max(1, int(ni * a.scale)), max(1, int(nr * a.scale))
    data = synth.generate(nu, ni, nr)
    (tu, ti, tr), _ = data.split()
    p = L.default_params()
    p.num_factors, p.num_blocks, p.iterations, p.seed = k, nb, a.epochs, 0
    p.mode = L.MODE_FAST_F32 if a.mode == "fast" else L.MODE_DETERMINISTIC_F64
    p.online_learning_rate = 0.01
    flav = {"flink": L.ONLINE_NEXT_FACTORS, "ps": L.ONLINE_DELTA, "spark": L.ONLINE_SPARK_SWEEP}[a.flavour]
    with mfhip.Context(p) as ctx:
        t0 = time.time()
        ctx.fit(tu, ti, tr)
        ctx.sync()
        t_fit = time.time() - t0
        stream = synth.generate(nu, ni, a.batch * a.batches, seed=99, test_fraction=0.0)
        rates, levels = [], []
        for b in range(a.batches):
            s = slice(b * a.batch, (b + 1) * a.batch)
            ctx.reset_stats()
            t0 = time.perf_counter()
            ctx.online_update(stream.u[s], stream.i[s], stream.r[s], flav, a.partitions)
            ctx.sync()
            dt = time.perf_counter() - t0
            rates.append(a.batch / dt)
            levels.append(ctx.stats()["levels"])
            print(f"batch {b}: {a.batch / dt / 1e6:.1f} M ratings/s ({dt * 1e3:.1f} ms, {levels[-1]} levels)", flush=True)
    rec = {"config": a.config, "scale": a.scale, "rank": k, "mode": a.mode, "flavour": a.flavour,
           "offline_epochs": a.epochs, "offline_fit_s": round(t_fit, 2), "batch": a.batch, "batches": a.batches,
           "ratings_per_s_median": float(np.median(rates)), "ratings_per_s_min": float(min(rates)),
           "levels_median": float(np.median(levels)), "target_ratings_per_s": 10e6,
           "timing": "end to end per micro-batch: host id lookup, dependency-level plan, H2D, kernels, sync"}
    print(json.dumps(rec), flush=True)
    if a.out:
        json.dump(rec, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
