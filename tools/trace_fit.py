#!/usr/bin/env python3
"""Fit per-wave duration = startup + steps * per_step from an MFHIP_WAVE_TRACE dump, per wave kind,
and compare the sum of sub-step spans with the sum of the longest waves (launch gaps / skew)."""
import sys

import numpy as np

a = np.loadtxt(sys.argv[1], dtype=np.int64)
dur = (a[:, 7] - a[:, 6]) * 10.0
for kind in (1, 2):
    m = (a[:, 5] == kind) & (a[:, 4] > 0)
    if m.sum() < 10:
        continue
    A = np.stack([np.ones(m.sum()), a[m, 4]], 1)
    coef, *_ = np.linalg.lstsq(A, dur[m], rcond=None)
    print(f"kind {kind}: waves {m.sum()}, startup {coef[0]:.0f} ns, per step {coef[1]:.1f} ns, "
          f"median steps {np.median(a[m, 4]):.0f}")
sub = a[:, 1] * 100000 + a[:, 2] + a[:, 0] * 10**9
spans, crit, first_start_lag, startlag = [], [], [], []
keys = np.unique(sub)
prev_end = None
for key in keys:
    w = a[sub == key]
    spans.append((w[:, 7].max() - w[:, 6].min()) * 10.0)
    crit.append(((w[:, 7] - w[:, 6]) * 10.0).max())
    startlag.append((w[:, 6].max() - w[:, 6].min()) * 10.0)
    if prev_end is not None:
        first_start_lag.append((w[:, 6].min() - prev_end) * 10.0)
    prev_end = w[:, 7].max()
spans, crit = np.array(spans), np.array(crit)
print(f"sub-steps {len(keys)}: sum span {spans.sum()/1e6:.2f} ms, sum longest wave {crit.sum()/1e6:.2f} ms, "
      f"median start skew {np.median(startlag):.0f} ns, median gap between launches {np.median(first_start_lag):.0f} ns")
