#!/usr/bin/env python3
"""Hot-item replica diagnosis: fit a scaled NFLX-shaped synthetic epoch by epoch and report
NaN rows and RMSE per epoch for the given item_split and env knobs."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-recommendation_amd"))
import mfhip  # noqa: E402
from mfhip import _lib as L, synth  # noqa: E402

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 0.1
split = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
epochs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
nu, ni, nr, k, nb = synth.CONFIGS["NFLX"]
d = synth.generate(int(nu * scale), int(ni * scale), int(nr * scale))
(tu, ti, tr), (eu, ei, er) = d.split()
p = L.default_params()
p.num_factors, p.num_blocks, p.seed, p.has_seed, p.iterations = k, nb, 0, 1, epochs
p.mode = L.MODE_FAST_F32
os.environ["MFHIP_ITEM_SPLIT"] = str(split)
ctx = mfhip.Context(p)
ctx.prepare(tu, ti, tr)
for e in range(epochs):
    for s in range(nb):
        ctx.run(1)
        _, itf = ctx.factors(L.SIDE_ITEM)
        _, uf = ctx.factors(L.SIDE_USER)
        bi, bu = np.isnan(itf).any(1).sum(), np.isnan(uf).any(1).sum()
        if bi or bu:
            print(f"epoch {e} superstep {s}: NaN item rows {bi} user rows {bu}", flush=True)
            sys.exit(1)
    rm, _ = ctx.rmse(eu, ei, er)
    print(f"epoch {e}: rmse {rm:.6f} max|I| {np.abs(itf).max():.3g} max|U| {np.abs(uf).max():.3g}", flush=True)
