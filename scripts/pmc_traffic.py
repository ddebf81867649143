#!/usr/bin/env python3
"""Turn rocprofv3 --pmc counter CSVs into per-launch HBM traffic of the quantize kernel.

gfx950 corrections (MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7):
  * FETCH_SIZE and WRITE_SIZE are in KiB;
  * FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced streaming read
    (16 B/lane loads, which is what the kernel issues) -> doubled;
  * WRITE_SIZE is exact for 16-B/lane stores; the kernel's 4-B/lane qweight stores are
    uncalibrated (noted in the output).
Usage: pmc_traffic.py --fetch dirA --write dirB --key llama3-70b.b4.asym.packed [--out profiles/round2/pmc_traffic.json]
"""
import argparse
import csv
import glob
import json
import os
import statistics

KERNEL = "awq_fast_kernel"


def read_counter(d, name):
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if KERNEL not in row.get("Kernel_Name", ""):
                    continue
                if row.get("Counter_Name") != name:
                    continue
                key = row.get("Dispatch_Id")
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--algo-bytes", type=float, default=None)
    ap.add_argument("--commit", default=None, help="commit the counters were measured on")
    ap.add_argument("--date", default=None)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "round3", "pmc_traffic.json"))
    a = ap.parse_args()
    fetch = read_counter(a.fetch, "FETCH_SIZE")
    write = read_counter(a.write, "WRITE_SIZE")
    if not fetch or not write:
        raise SystemExit(f"no counter rows for {KERNEL}: fetch={len(fetch)} write={len(write)}")
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    rd = f_kib * 1024 * 2
    wr = w_kib * 1024
    rec = {"hbm_bytes_per_launch": rd + wr, "read_bytes": rd, "write_bytes": wr,
           "fetch_size_kib_median": f_kib, "write_size_kib_median": w_kib, "dispatches": [len(fetch), len(write)],
           "correction": "FETCH_SIZE x2 (gfx950 half-count of 16B/lane streaming reads); WRITE_SIZE as reported"}
    rec["commit"], rec["date"] = a.commit, a.date
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    rec["kernel_source_sha256"] = bench.kernel_source_hash()   # bench.py marks the record stale when it changes
    if a.algo_bytes:
        rec["algorithmic_bytes_per_launch"] = a.algo_bytes
        rec["traffic_over_algorithmic"] = (rd + wr) / a.algo_bytes
    data = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            data = json.load(f)
    data[a.key] = rec
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(json.dumps({a.key: rec}))


if __name__ == "__main__":
    main()
