#!/usr/bin/env python3
"""rocprofv3 kernel trace -> durations of the bench's timed window (the last --steps
launches of the kernel) next to the whole-run average the --stats summary reports, so the
bench line's HIP-event kernel time can be checked against the profiler on the same window.

  python scripts/trace_window.py gpurun_out/r61/trace/bench_kernel_trace.csv --steps 1000
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--kernel", default="awq_fast_kernel")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    ts = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    d = [(e - s) / 1e3 for s, e in ts]
    w = d[-a.steps:]
    span = (ts[-1][1] - ts[-len(w)][0]) / 1e3
    print(json.dumps({"launches": len(d), "all_mean_us": round(sum(d) / len(d), 2),
                      "window_launches": len(w), "window_mean_us": round(sum(w) / len(w), 2),
                      "window_median_us": round(sorted(w)[len(w) // 2], 2),
                      "window_span_per_launch_us": round(span / len(w), 2)}))


if __name__ == "__main__":
    main()
