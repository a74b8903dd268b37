#!/usr/bin/env python3
"""Summarise an MFHIP_WAVE_TRACE dump (per wave: shard sm t wave steps cells start end, 100 MHz).

Per sub-step: span (first start .. last end), the longest wave's steps and ns/step, and the
median ns/step of the other waves; then the sum of spans against the sum of the longest
waves' busy time (the rest is launch gap and tail)."""
import sys

import numpy as np

a = np.loadtxt(sys.argv[1], dtype=np.int64)
if a.ndim == 1:
    a = a[None, :]
sub = a[:, 1] * 100000 + a[:, 2]
tot_span = tot_crit = 0.0
rows = []
for key in np.unique(sub):
    w = a[sub == key]
    st, en = w[:, 6], w[:, 7]
    span = (en.max() - st.min()) * 10.0  # ns
    dur = (en - st) * 10.0
    crit = np.argmax(en)
    steps = w[:, 4]
    nsps = dur / np.maximum(steps, 1)
    rows.append((key // 100000, key % 100000, len(w), span / 1e3, int(steps[crit]), nsps[crit], float(np.median(nsps)),
                 float(dur.mean() / 1e3), int(steps.max())))
    tot_span += span
    tot_crit += dur[crit]
print("sm t waves span_us crit_steps crit_ns/step median_ns/step mean_wave_us max_steps")
for r in rows[:: max(1, len(rows) // 24)]:
    print("%2d %3d %5d %8.1f %6d %8.1f %8.1f %8.1f %6d" % r)
arr = np.array([r[3:] for r in rows], dtype=float)
print(f"sub-steps {len(rows)}  sum span {tot_span/1e6:.2f} ms  sum critical-wave busy {tot_crit/1e6:.2f} ms")
print(f"median crit ns/step {np.median(arr[:,2]):.1f}  median other ns/step {np.median(arr[:,3]):.1f}  "
      f"mean crit steps {arr[:,1].mean():.1f}")
