#!/usr/bin/env python3
"""Average SQ counters per launch of each kernel in a rocprofv3 --pmc counter_collection.csv."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0][-60:]
    acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[name].add(r["Dispatch_Id"])
for name, d in acc.items():
    n = len(cnt[name])
    print(name, "launches", n)
    for c, v in sorted(d.items()):
        print(f"  {c:24s} {v / n:16.1f}")
