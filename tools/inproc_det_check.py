import os, sys, numpy as np
sys.path.insert(0, "large-scale-recommendation_amd")
import mfhip
from mfhip import _lib as L
d = mfhip.synth.config("YAHOO", 0.05)
(tu, ti, tr), _ = d.split()
outs = []
for rep in range(2):
    p = L.default_params()
    p.num_factors, p.num_blocks, p.iterations, p.seed, p.has_seed = 256, 8, 1, 5, 1
    p.mode = L.MODE_FAST_F32
    p.fast_waves = -16
    with mfhip.Context(p, devices=[0] * 8) as ctx:
        ctx.fit(tu, ti, tr)
        outs.append((ctx.factors(0)[1], ctx.factors(1)[1]))
print("in-process 8 shards deterministic:", np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1]),
      float(np.abs(outs[0][0] - outs[1][0]).max()))
