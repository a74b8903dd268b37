#!/usr/bin/env python3
"""Superstep-time model of the fast pair schedule: one launch per sub-step (global barrier) vs a
systolic persistent launch (cell (g,t) waits only for (g,t-1) and (g+1,t-1)).  Cell cost =
startup + pairs * per_pair by kind (fit from a wave trace, tools/trace_fit.py)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-recommendation_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="NFLX")
ap.add_argument("--groups", type=int, default=128)
ap.add_argument("--scale", type=float, default=1.0)
ap.add_argument("--gap", type=float, default=2960.0, help="ns between launches (sub-step model)")
ap.add_argument("--mixed", default="2900,215", help="startup_ns,per_pair_ns of mixed cells")
ap.add_argument("--single", default="2400,155", help="startup_ns,per_pair_ns of single-item cells")
ap.add_argument("--handoff", default="1000,2000,3000", help="systolic per-cell transition ns values")
a = ap.parse_args()

import ctypes as C
from mfhip import _lib as L, synth

nu, ni, nr, k, nb = synth.CONFIGS[a.config]
d = synth.generate(int(nu * a.scale), int(ni * a.scale), int(nr * a.scale))
(tu, ti, tr), _ = d.split()
n = len(tu)
blk = np.empty(n, np.int32); sub = np.empty(n, np.int32); grp = np.empty(n, np.int32); pos = np.empty(n, np.int64)
win = C.c_int32()
L.lib().mf_fast_plan_window(k, C.byref(win))
P = lambda x, t: x.ctypes.data_as(C.POINTER(t))
rc = L.lib().mf_debug_fast_schedule(P(tu, C.c_int32), P(ti, C.c_int32), n, nb, 0, a.groups, 0, win.value, k,
                                    P(blk, C.c_int32), P(sub, C.c_int32), P(grp, C.c_int32), P(pos, C.c_int64))
assert rc == 0, L.lib().mf_last_error()
G = a.groups
cell = (blk.astype(np.int64) * G + sub) * G + grp
ncell = nb * nb * G * G
length = np.zeros(ncell, np.int64)
np.maximum.at(length, cell, pos + 1)
# distinct items per cell
key = cell * (1 << 32) + ti.astype(np.int64) - ti.min()
uniq = np.unique(key)
nitems = np.bincount(uniq >> 32, minlength=ncell)
pairs = (length + 1) // 2
ms, mp = map(float, a.mixed.split(",")); ss, sp = map(float, a.single.split(","))
single = nitems == 1
cost_work = np.where(single, sp, mp) * pairs
startup = np.where(single, ss, ms)
cost_work = cost_work.reshape(nb, nb, G, G)  # [ub, ib, t, g]
startup = startup.reshape(nb, nb, G, G)
has = (pairs > 0).reshape(nb, nb, G, G)

barrier = 0.0
syst = {float(h): 0.0 for h in a.handoff.split(",")}
for s in range(1, nb + 1):
    blocks = [(p, (p + s - 1) % nb) for p in range(nb)]
    for t in range(G):
        barrier += max(float((cost_work[p, q, t] + startup[p, q, t] * has[p, q, t]).max()) for p, q in blocks) + a.gap
    for h in syst:
        worst = 0.0
        for p, q in blocks:
            c = cost_work[p, q] + h * has[p, q]  # [t, g]
            fin = np.zeros(G)
            for t in range(G):
                start = np.maximum(fin, np.roll(fin, -1)) if t > 0 else fin
                fin = start + c[t]
            worst = max(worst, float(fin.max()))
        syst[h] += worst + a.gap
print(f"{a.config} G={G}: cells {int(has.sum())}, single-item {int((single & (pairs > 0)).sum())}")
print(f"  sub-step launches: {barrier / 1e6:.2f} ms/epoch")
for h, v in syst.items():
    print(f"  systolic, {h:.0f} ns per cell hand-off: {v / 1e6:.2f} ms/epoch")
