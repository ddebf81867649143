#!/usr/bin/env python3
"""Average kernel duration per (kernel, grid) from a rocprofv3 kernel_trace.csv — one line per
distinct launch shape (the --stats summary averages all shapes of a kernel together).

  python scripts/trace_avg.py <kernel_trace.csv> [name-regex]
"""
import csv
import json
import re
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if not rx.search(r["Kernel_Name"]):
            continue
        name = r["Kernel_Name"]
        m = re.search(r"<([^<>]*(?:<[^<>]*>[^<>]*)*)>", name)
        short = name.split("(")[0].split("::")[-1].split("<")[0] + ("<" + m.group(1) + ">" if m else "")
        key = (short, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
        acc[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for (k, g, w), v in sorted(acc.items()):
        v.sort()
        print(json.dumps({"kernel": k, "grid": g, "block": w, "launches": len(v), "avg_us": round(sum(v) / len(v) / 1e3, 2),
                          "median_us": round(v[len(v) // 2] / 1e3, 2), "min_us": round(v[0] / 1e3, 2)}))


if __name__ == "__main__":
    main()
