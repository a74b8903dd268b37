#!/usr/bin/env python3
"""Does a fast-mode fit repeat itself?  Fit once, then restart (mf_dsgd_restart) and rerun the same
epochs several times; every rerun must reproduce the first fit's factors bit for bit (the
systolic sweep has no atomics and a fixed plan).

    python tools/repeat_check.py --config YAHOO --scale 0.05 --epochs 10 --reruns 3 [--knobs pair_sys=0]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-recommendation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="YAHOO")
    ap.add_argument("--scale", type=float, default=0.05)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--reruns", type=int, default=3)
    ap.add_argument("--knobs", default=None, help="MFHIP_TEST for this run")
    ap.add_argument("--k", type=int, default=0, help="rank (default: the config's)")
    a = ap.parse_args()
    if a.knobs:
        os.environ["MFHIP_TEST"] = a.knobs
    import mfhip
    from mfhip import _lib as L
    d = mfhip.synth.config(a.config, a.scale)
    (tu, ti, tr), (eu, ei, er) = d.split()
    del d
    _, _, _, k, nb = mfhip.synth.CONFIGS[a.config]
    k = a.k or k
    p = L.default_params()
    p.num_factors, p.num_blocks, p.iterations, p.seed, p.mode = k, nb, a.epochs, 0, L.MODE_FAST_F32
    with mfhip.Context(p) as ctx:
        ctx.fit(tu, ti, tr)
        r0, _ = ctx.rmse(eu, ei, er)
        u0, i0 = ctx.factors(L.SIDE_USER)[1], ctx.factors(L.SIDE_ITEM)[1]
        same = 0
        for x in range(a.reruns):
            ctx.restart()
            ctx.run(a.epochs * nb)
            r, _ = ctx.rmse(eu, ei, er)
            u, i = ctx.factors(L.SIDE_USER)[1], ctx.factors(L.SIDE_ITEM)[1]
            du = int(np.sum(np.any(u != u0, axis=1)))
            di = int(np.sum(np.any(i != i0, axis=1)))
            same += du == 0 and di == 0
            print(f"rerun {x + 1}: rmse {r:.9f} vs {r0:.9f}; differing user rows {du}, item rows {di}", flush=True)
    print(f"REPEAT {a.config}@{a.scale:g} k={k} knobs={a.knobs}: {same} of {a.reruns} reruns identical", flush=True)


if __name__ == "__main__":
    main()
