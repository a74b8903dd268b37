#!/usr/bin/env python3
"""Summarise an MFHIP_WAVE_TRACE dump of the systolic pair sweep (rows: shard sm t wave steps kind
start end, one per cell, 100 MHz): per-kind cell cost fit, the gaps between a wave's consecutive
cells (neighbour wait + hand-off), and each superstep's span."""
import collections
import sys

import numpy as np

a = np.loadtxt(sys.argv[1], dtype=np.int64, ndmin=2)
a = a[a[:, 6] > 0]
clk = a.shape[1] > 8  # 9th column: shader-clock cycles of the cell (s_memtime)
dur = (a[:, 7] - a[:, 6]) * 10.0
for kind in (1, 2):
    m = (a[:, 5] == kind) & (a[:, 4] > 0)
    if m.sum() < 10:
        continue
    A = np.stack([np.ones(m.sum()), a[m, 4]], 1)
    coef, *_ = np.linalg.lstsq(A, dur[m], rcond=None)
    print(f"kind {kind}: cells {m.sum()}, fixed {coef[0]:.0f} ns, per pair {coef[1]:.1f} ns, median pairs {np.median(a[m, 4]):.0f}")
e = a[a[:, 4] == 0]
print(f"empty cells {len(e)}, median duration {np.median((e[:, 7] - e[:, 6]) * 10.0) if len(e) else 0:.0f} ns")
order = np.lexsort((a[:, 2], a[:, 3], a[:, 1], a[:, 0]))
b = a[order]
same = (b[1:, 0] == b[:-1, 0]) & (b[1:, 1] == b[:-1, 1]) & (b[1:, 3] == b[:-1, 3])
gap = (b[1:, 6] - b[:-1, 7])[same] * 10.0
print(f"gap between a wave's cells: median {np.median(gap):.0f} ns, p10 {np.percentile(gap, 10):.0f}, "
      f"p90 {np.percentile(gap, 90):.0f}, mean {gap.mean():.0f}")
tot = 0.0
for sm in np.unique(a[:, 1]):
    w = a[a[:, 1] == sm]
    span = (w[:, 7].max() - w[:, 6].min()) * 10.0
    busy = np.zeros(0)
    tot += span
    waves = np.unique(w[:, 3])
    per_wave = [((w[w[:, 3] == x, 7] - w[w[:, 3] == x, 6]) * 10.0).sum() for x in waves]
    xm = waves[int(np.argmax(per_wave))]
    print(f"superstep {sm}: span {span / 1e3:.0f} us, busiest wave {xm} busy {max(per_wave) / 1e3:.0f} us "
          f"({int(w[w[:, 3] == xm, 4].sum())} pairs), median wave busy {np.median(per_wave) / 1e3:.0f} us")
    # the busiest wave's time split: in cells (fixed cost + pairs) and between cells (hand-off waits)
    c = w[w[:, 3] == xm]
    c = c[np.argsort(c[:, 2])]
    d = (c[:, 7] - c[:, 6]) * 10.0
    g = (c[1:, 6] - c[:-1, 7]) * 10.0
    pairs = c[:, 4].sum()
    nz = c[:, 4] > 0
    fit = np.linalg.lstsq(np.stack([np.ones(nz.sum()), c[nz, 4]], 1), d[nz], rcond=None)[0] if nz.sum() > 2 else [0, 0]
    print(f"    busiest wave: {len(c)} cells (kinds {sorted(set(c[:, 5].tolist()))}), first start +"
          f"{(c[0, 6] - w[:, 6].min()) * 10.0 / 1e3:.1f} us, in cells {d.sum() / 1e3:.0f} us = {d.sum() / max(pairs, 1):.0f} "
          f"ns/pair (fit: {fit[0]:.0f} ns/cell + {fit[1]:.1f} ns/pair), between cells {g.sum() / 1e3:.0f} us "
          f"(median {np.median(g) if len(g) else 0:.0f} ns)"
          + (f", shader clock {c[:, 8].sum() / max(d.sum(), 1):.2f} GHz vs all waves "
             f"{w[:, 8].sum() / max(((w[:, 7] - w[:, 6]) * 10.0).sum(), 1):.2f} GHz, {c[:, 8].sum() / max(pairs, 1):.0f} "
             f"cycles/pair" if clk else ""))
    if a.shape[1] > 9:  # 10th column: XCC_ID << 32 | HW_ID of the wave (the first cell's)
        loc = {}
        for x in waves:
            h = int(w[w[:, 3] == x, 9][0])
            xcc, hw = h >> 32, h & 0xFFFFFFFF
            cu = (xcc & 0xF, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xF)  # xcc, se, sh, cu
            loc[x] = (cu, (hw >> 4) & 3)
        cu_m, simd_m = loc[xm]
        same_cu = [x for x in waves if x != xm and loc[x][0] == cu_m]
        same_simd = [x for x in same_cu if loc[x][1] == simd_m]
        per_simd = collections.Counter(loc.values())
        busy = dict(zip(waves, per_wave))
        print(f"    placement: busiest wave on xcc/se/sh/cu {cu_m} simd {simd_m}; {len(same_cu)} other waves on its CU "
              f"(busy {[round(busy[x] / 1e3) for x in same_cu]} us), {len(same_simd)} on its SIMD; SIMDs holding 1/2/3+ "
              f"waves: {sum(v == 1 for v in per_simd.values())}/{sum(v == 2 for v in per_simd.values())}/"
              f"{sum(v >= 3 for v in per_simd.values())}")
print(f"sum of superstep spans {tot / 1e6:.2f} ms")
