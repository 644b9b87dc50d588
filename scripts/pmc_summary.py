#!/usr/bin/env python3
"""Summarise a rocprofv3 counter_collection.csv: per kernel (k_* name), per dispatch sums of each
counter, averaged over dispatches.  Usage: pmc_summary.py <csv> [name-filter]"""
import collections
import csv
import re
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> ctr -> sum
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+)(<[^>(]*>)?", r["Kernel_Name"])
    if not m or "cusz" not in r["Kernel_Name"]:
        continue
    name = m.group(1) + (m.group(2) or "")
    rows[(name, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for (name, _), d in rows.items():
    for c, v in d.items():
        acc[name][c].append(v)
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for name, d in acc.items():
    if flt in name:
        n = len(next(iter(d.values())))
        print(f"{name} (x{n}): " + ", ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(d.items())))
