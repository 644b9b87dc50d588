#!/usr/bin/env python3
"""Average rocprofv3 counter values per dispatch for kernels matching a substring.
usage: pmc_kernel.py SUBSTR DIR [DIR ...]   (each DIR holds a run_counter_collection.csv)"""
import csv
import glob
import os
import sys

sub = sys.argv[1]
acc = {}
for d in sys.argv[2:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            acc.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for k in sorted(acc):
    v = list(acc[k].values())
    print(f"{k:36s} {sum(v) / len(v):16.1f}   (n={len(v)})")
