#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/: kernel stats + PMC HBM traffic per launch.

usage: scripts/prof_summary.py TAG STATS_DIR [PMC_FETCH_DIR PMC_WRITE_DIR]
HBM bytes per launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024: on gfx950 FETCH_SIZE reports half
the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, HBM section); the x2 is
exact for 16-B-per-lane streams and an over-estimate for narrower reads (noted per kernel).
"""
import csv
import json
import re
import os
import shutil
import sys

tag, stats = sys.argv[1], sys.argv[2]
out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
os.makedirs(out, exist_ok=True)
src = os.path.join(stats, "run_kernel_stats.csv")
shutil.copy(src, os.path.join(out, f"{tag}_kernel_stats.csv"))
rows = list(csv.DictReader(open(src)))
summary = {}
for r in rows:
    name = r["Name"]
    if "cusz_amd" not in name:
        continue
    short = re.search(r"\b(k_\w+)", name).group(1)
    summary[short] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                      "max_ns": float(r["MaxNs"]), "full_name": name[:160]}
if len(sys.argv) > 4:
    for d, cname in ((sys.argv[3], "FETCH_SIZE"), (sys.argv[4], "WRITE_SIZE")):
        f = os.path.join(d, "run_counter_collection.csv")
        rows_pmc = list(csv.DictReader(open(f)))
        keep = [r for r in rows_pmc if "cusz_amd" in r["Kernel_Name"]]
        if keep:  # only our kernels' rows are kept (the datagen torch kernels are noise)
            with open(os.path.join(out, f"{tag}_pmc_{cname.lower()}.csv"), "w", newline="") as fo:
                w = csv.DictWriter(fo, fieldnames=list(keep[0].keys()))
                w.writeheader()
                w.writerows(keep)
        acc = {}
        for r in rows_pmc:
            if "cusz_amd" not in r["Kernel_Name"] or r["Counter_Name"] != cname:
                continue
            short = re.search(r"\b(k_\w+)", r["Kernel_Name"]).group(1)
            acc.setdefault(short, []).append(float(r["Counter_Value"]))
        for k, v in acc.items():
            summary.setdefault(k, {})[cname.lower() + "_kb"] = sum(v) / len(v)
    for k, s in summary.items():
        if "fetch_size_kb" in s and "write_size_kb" in s:
            s["hbm_bytes_per_launch"] = int((2 * s["fetch_size_kb"] + s["write_size_kb"]) * 1024)
json.dump(summary, open(os.path.join(out, f"{tag}_summary.json"), "w"), indent=1)
json.dump(summary, open(os.path.join(out, "pmc_latest.json"), "w"), indent=1)
for k, s in sorted(summary.items(), key=lambda kv: -kv[1].get("avg_ns", 0)):
    print(f"{k:24s} calls={s.get('calls')} avg={s.get('avg_ns', 0)/1e3:9.1f} us  "
          f"hbm/launch={s.get('hbm_bytes_per_launch', 0)/2**20:9.1f} MiB")
