#!/usr/bin/env python3
"""Write the training split of a bench config as raw arrays for tools/probe/plan_probe."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "large-scale-recommendation_amd"))
from mfhip import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "NFLX"
out = sys.argv[2] if len(sys.argv) > 2 else "/tmp"
nu, ni, nr, k, nb = synth.CONFIGS[cfg]
(tu, ti, tr), _ = synth.generate(nu, ni, nr).split()
tu.tofile(f"{out}/probe_u.bin"); ti.tofile(f"{out}/probe_i.bin"); tr.tofile(f"{out}/probe_r.bin")
print(cfg, len(tu), "ratings", "k", k, "n", nb)
