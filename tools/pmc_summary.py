#!/usr/bin/env python3
"""Summarise rocprofv3 output of bench.py into a per-launch HBM traffic record.

    python tools/pmc_summary.py --stats gpurun_out/rocprof_kt/kt_kernel_stats.csv \
        --fetch gpurun_out/rocprof_fetch/fetch_counter_collection.csv \
        --write gpurun_out/rocprof_write/write_counter_collection.csv \
        --kernel k_fast_substep --config NFLX --mode fast --rank 128 --groups 124 \
        --out profiles/r01_traffic_NFLX_fast.json

FETCH_SIZE / WRITE_SIZE are reported in KiB.  On gfx950 FETCH_SIZE counts half of the bytes of
wide reads (MI355X_MICROARCH.md, HBM section), so the read side is doubled; WRITE_SIZE is
taken as is.  The counters were collected in two separate --pmc passes (TCC block budget).
"""
import argparse
import csv
import json


def kernel_match(name, kernel):
    """rocprof kernel names are demangled signatures: match the template name exactly, or, for a
    kernel given with its template arguments ("k_det_sweep_split<2, 1>"), that instance only."""
    if "<" in kernel:
        return kernel.replace(" ", "") + "(" in name.replace(" ", "")
    return f"{kernel}<" in name or name.split("(")[0].endswith(kernel)


def counter(path, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if kernel_match(r["Kernel_Name"], kernel)]
    return len(vals), (sum(vals) / len(vals) if vals else 0.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="k_fast_substep")
    ap.add_argument("--config", default="NFLX")
    ap.add_argument("--mode", default="fast")
    ap.add_argument("--rank", type=int, default=128)
    ap.add_argument("--groups", type=int, default=0)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    st = [r for r in csv.DictReader(open(a.stats)) if kernel_match(r["Name"], a.kernel)]
    assert st, f"kernel {a.kernel} not in {a.stats}"
    nf, fetch_kib = counter(a.fetch, a.kernel)
    nw, write_kib = counter(a.write, a.kernel)
    fetch = 2.0 * fetch_kib * 1024.0
    write = write_kib * 1024.0
    rec = {"kernel": a.kernel, "config": a.config, "mode": a.mode, "rank": a.rank, "groups": a.groups,
           "calls": int(st[0]["Calls"]), "avg_ns": float(st[0]["AverageNs"]),
           "pmc_launches": [nf, nw], "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "bytes_per_launch": fetch + write,
           "correction": "FETCH_SIZE x 1024 x 2 (gfx950 half-count), WRITE_SIZE x 1024"}
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
