#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection CSVs: per kernel name, median per-dispatch value
of every counter.  Usage: pmc_summary.py DIR > summary.json"""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
per = {}
for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row.get("Kernel_Name", "?")[:120]
            key = (k, row.get("Dispatch_Id"), row.get("Counter_Name"))
            per[key] = per.get(key, 0.0) + float(row.get("Counter_Value", 0) or 0)
agg = {}
for (k, disp, cname), v in per.items():
    agg.setdefault(k, {}).setdefault(cname, []).append(v)
out = {k: {c: {"median": statistics.median(v), "n": len(v)} for c, v in cs.items()} for k, cs in agg.items()}
print(json.dumps(out, indent=1))
