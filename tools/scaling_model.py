#!/usr/bin/env python3
"""Strong-scaling model of the NFLX fast sweep on 1/2/4/8 GPUs (rank mode, n = 8) from the plan
(tools/probe/plan_probe ... scale: per rank, superstep and wave its cells, single-run pairs and
mixed pairs) and per-pair / per-cell costs measured in wave traces (tools/sys_trace.py).

A superstep on a rank lasts as long as its busiest wave (the systolic hand-offs add ~3% on the
busiest wave in the traces, folded into the per-cell cost); an epoch is the sum over supersteps of
the slowest rank, plus one item-block ring step per superstep.  Two cost sets: 'loaded' (the
in-situ costs of the one-GPU run, every SIMD busy) and 'isolated' (the one-wave chain alone on the
chip, the best a lightly loaded GPU can do).

    python tools/scaling_model.py /tmp/scale_probe.txt [t_run_loaded t_mix_loaded t_run_iso cell_ns]
"""
import collections
import gzip
import sys

path = sys.argv[1]
t_run_l = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0   # ns per single-run pair, loaded (wave trace)
t_mix_l = float(sys.argv[3]) if len(sys.argv) > 3 else 212.0   # ns per mixed pair, loaded
t_run_i = float(sys.argv[4]) if len(sys.argv) > 4 else 127.6   # ns per single-run pair, isolated chain
cell_ns = float(sys.argv[5]) if len(sys.argv) > 5 else 2500.0  # per non-empty cell: fill, drain, hand-off
ring_us = 20.0  # one item-block send/recv per superstep (1.1 MB over one xGMI link + launch), not overlapped at c = 1

waves = collections.defaultdict(list)  # (G, rank, sm) -> [(cells, run, mix)]
for line in (gzip.open(path, "rt") if path.endswith(".gz") else open(path)):
    if not line.startswith("SCALE"):
        continue
    f = line.split()
    G, rank, sm = int(f[2]), int(f[4]), int(f[6])
    waves[(G, rank, sm)].append((int(f[10]), int(f[12]), int(f[14])))

print("| GPUs | busiest-wave pairs per superstep (max over ranks, mean over supersteps) | epoch, loaded costs (ms) | "
      "epoch, isolated costs (ms) | speed-up vs 1 GPU (loaded / isolated) |")
print("|---|---|---|---|---|")
base = None
for G in sorted({k[0] for k in waves}):
    ep_l = ep_i = 0.0
    pairs = []
    for sm in sorted({k[2] for k in waves if k[0] == G}):
        worst_l = worst_i = 0.0
        wp = 0
        for rank in range(G):
            for cells, run, mix in waves.get((G, rank, sm), []):
                tl = cells * cell_ns + run * t_run_l + mix * t_mix_l
                ti = cells * cell_ns + (run * t_run_i + mix * t_mix_l * t_run_i / t_run_l)
                if tl > worst_l:
                    worst_l, wp = tl, run + mix
                worst_i = max(worst_i, ti)
        pairs.append(wp)
        ep_l += worst_l + (ring_us * 1e3 if G > 1 else 0.0)
        ep_i += worst_i + (ring_us * 1e3 if G > 1 else 0.0)
    if base is None:
        base = ep_l
    print(f"| {G} | {sum(pairs) / len(pairs):.0f} | {ep_l / 1e6:.2f} | {ep_i / 1e6:.2f} | "
          f"{base / ep_l:.2f} / {base / ep_i:.2f} |")
