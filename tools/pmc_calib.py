#!/usr/bin/env python3
"""Calibrate FETCH_SIZE / WRITE_SIZE against known bytes (tools/micro/fetch_calib.hip).

    python tools/pmc_calib.py --cases fetch_calib.txt --fetch <fetch counter_collection.csv> \
        --write <write counter_collection.csv> --out profiles/r06_fetch_calib.json

Pairs every dispatch of the micro benchmark with its known read / write bytes and prints the
ratio counter_bytes / known_bytes (counters in KiB, raw, no correction applied): a read ratio of
0.5 is the gfx950 half-count MI355X_MICROARCH.md documents for 16-B/lane streaming reads, 1.0 an
exact count.  The sweeps' PMC summaries (tools/pmc_summary.py) double FETCH_SIZE; this says whether
that holds for their 8-B/lane random-row accesses.
"""
import argparse
import csv
import json


def per_dispatch(path):
    """Counter value per dispatch, in dispatch order (rocprofv3 counter_collection.csv)."""
    rows = list(csv.DictReader(open(path)))
    key = "Dispatch_Id" if rows and "Dispatch_Id" in rows[0] else "Correlation_Id"
    acc = {}
    for r in rows:
        if "k_rows" not in r.get("Kernel_Name", "k_rows"):  # the benchmark's own kernels (not the memset)
            continue
        acc[int(r[key])] = acc.get(int(r[key]), 0.0) + float(r["Counter_Value"])
    return [acc[d] for d in sorted(acc)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    cases = [r for r in csv.DictReader(open(a.cases)) if r.get("case")]
    fetch, write = per_dispatch(a.fetch), per_dispatch(a.write)
    assert len(fetch) == len(cases) and len(write) == len(cases), (len(fetch), len(write), len(cases))
    out = []
    for c, f, w in zip(cases, fetch, write):
        rd, wr = float(c["read_bytes"]), float(c["write_bytes"])
        rec = {"case": c["case"], "read_bytes": rd, "write_bytes": wr, "ms": float(c["ms"]),
               "fetch_bytes_raw": f * 1024.0, "write_bytes_raw": w * 1024.0,
               "fetch_ratio_raw": round(f * 1024.0 / rd, 4) if rd else None,
               "write_ratio_raw": round(w * 1024.0 / wr, 4) if wr else None}
        out.append(rec)
        print(json.dumps(rec))
    json.dump({"source": "tools/micro/fetch_calib.hip under rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE",
               "cases": out}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
