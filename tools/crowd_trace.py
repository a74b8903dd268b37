#!/usr/bin/env python3
"""Per-CU crowding view of an MFHIP_WAVE_TRACE dump (10 columns: shard sm t wave steps kind start end
clk place): waves per superstep, ns per pair in cells by the number of waves sharing the CU, and the
gaps between a wave's cells (neighbour waits), so a group-count change can be read as "steps got
slower" (crowding) or "waits grew" (systolic coupling)."""
import collections
import sys

import numpy as np

a = np.loadtxt(sys.argv[1], dtype=np.int64, ndmin=2)
a = a[a[:, 6] > 0]
dur = (a[:, 7] - a[:, 6]) * 10.0
print(f"supersteps {len(np.unique(a[:, 1]))}, waves per superstep "
      f"{np.mean([len(np.unique(a[a[:, 1] == s, 3])) for s in np.unique(a[:, 1])]):.0f}, cells {len(a)}, "
      f"median pairs per cell {np.median(a[:, 4]):.0f}")
for kind in (1, 2):
    acc = collections.defaultdict(lambda: [0.0, 0])
    for sm in np.unique(a[:, 1]):
        w = a[a[:, 1] == sm]
        d = dur[a[:, 1] == sm]
        cu_of = {}
        for x in np.unique(w[:, 3]):
            h = int(w[w[:, 3] == x, 9][0])
            xcc, hw = h >> 32, h & 0xFFFFFFFF
            cu_of[x] = (xcc & 0xF, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xF)
        per_cu = collections.Counter(cu_of.values())
        m = (w[:, 5] == kind) & (w[:, 4] > 0)
        for row, t in zip(w[m], d[m]):
            n = per_cu[cu_of[row[3]]]
            acc[n][0] += t
            acc[n][1] += row[4]
    for n in sorted(acc):
        t, p = acc[n]
        print(f"kind {kind}: waves on the CU {n}: {t / max(p, 1):.1f} ns per pair in cells ({p} pairs)")
order = np.lexsort((a[:, 2], a[:, 3], a[:, 1], a[:, 0]))
b = a[order]
same = (b[1:, 0] == b[:-1, 0]) & (b[1:, 1] == b[:-1, 1]) & (b[1:, 3] == b[:-1, 3])
gap = (b[1:, 6] - b[:-1, 7])[same] * 10.0
fixed = np.linalg.lstsq(np.stack([np.ones(len(a)), a[:, 4]], 1), dur, rcond=None)[0]
print(f"cell fit {fixed[0]:.0f} ns + {fixed[1]:.1f} ns/pair; gap between a wave's cells: median {np.median(gap):.0f} ns, "
      f"mean {gap.mean():.0f}, p90 {np.percentile(gap, 90):.0f}; per wave: cells in "
      f"{np.mean([len(np.unique(b[(b[:, 1] == s) & (b[:, 3] == x), 2])) for s in np.unique(b[:, 1])[:1] for x in np.unique(b[b[:, 1] == s, 3])]):.0f}")
spans = [(a[a[:, 1] == s, 7].max() - a[a[:, 1] == s, 6].min()) * 10.0 for s in np.unique(a[:, 1])]
print(f"sum of superstep spans {sum(spans) / 1e6:.3f} ms")
