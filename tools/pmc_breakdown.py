#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection.csv files per counter over the dispatches of one kernel.

    python tools/pmc_breakdown.py --kernel k_sweep_pair_sys pass1/*counter_collection.csv pass2/... [--json out]

Prints one line per counter: the sum over the kernel's dispatches and the per-dispatch mean, then
derived ratios when their inputs are present (SQ wave-cycle shares, TA busy per CU-cycle).
"""
import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    tot = defaultdict(float)
    disp = defaultdict(set)
    for f in a.files:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if a.kernel not in name:
                continue
            c = r.get("Counter_Name")
            tot[c] += float(r["Counter_Value"])
            disp[c].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    out = {}
    for c in sorted(tot):
        n = max(1, len(disp[c]))
        out[c] = {"sum": tot[c], "dispatches": n, "per_dispatch": tot[c] / n}
        print(f"{c:34s} sum {tot[c]:14.4e}  dispatches {n:5d}  per dispatch {tot[c] / n:12.4e}")
    wc = tot.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA"):
            if c in tot:
                print(f"  {c} / SQ_WAVE_CYCLES = {tot[c] / wc:.3f}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
