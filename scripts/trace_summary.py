#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 trace database (rocpd sqlite written with -o <name>):
name, grid, calls, mean / min duration in us — for the export and other A/B runs.

  python scripts/trace_summary.py gpurun_out/<run>/prof/run_results.db [substring ...]
"""
import collections
import sqlite3
import sys


def main():
    db, subs = sys.argv[1], sys.argv[2:]
    c = sqlite3.connect(db)
    agg = collections.OrderedDict()
    for name, gx, gy, dur in c.execute("select name, grid_x, grid_y, duration from kernels order by start"):
        if subs and not any(s in name for s in subs):
            continue
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg.setdefault((short[-48:], gx, gy), []).append(dur / 1e3)
    for (name, gx, gy), d in agg.items():
        print(f"{name:48s} grid {gx:>8d} x {gy:<5d} calls {len(d):3d} mean {sum(d) / len(d):8.1f} min {min(d):8.1f}")


if __name__ == "__main__":
    main()
