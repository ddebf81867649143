#!/usr/bin/env python3
"""VALU work per unit of a VALU-bound kernel, from one rocprofv3 --pmc pass (kernel-trace
only) of a bench.py command, merged into the recorded file bench.py reads for its
`roofline.peak` (bound "valu"):

  valu_slots_per_unit      = (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) per dispatch / units
                             (issue slots: one per SIMD per quad-cycle; a slot issues one VALU
                             instruction or two of the dual-issue class; scripts/valu_classes.py)
  valu_slot_occupancy      = those slots / (dispatch quad-cycles x 1024 SIMDs)
                             (dispatch cycles = GRBM_GUI_ACTIVE / 8, summed over the 8 XCDs)
  dual_issued_instr_frac   = 2 x SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU
  valu_lane_instr_per_unit = SQ_INSTS_VALU x 64 / units (for reference)

  pmc_valu.py --pmc-dir DIR --kernel REGEX --units-per-dispatch U --key KEY --sources fast|act
              --out profiles/round5/pmc_valu.json [--commit C] [--kernel-us T]
"""
import argparse
import csv
import datetime
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def counters(pmc_dir, kernel_rx):
    rx = re.compile(kernel_rx)
    per = {}
    for path in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if not rx.search(row.get("Kernel_Name", "")):
                    continue
                key = (row.get("Dispatch_Id"), row.get("Counter_Name"))
                per[key] = per.get(key, 0.0) + float(row.get("Counter_Value", 0) or 0)
    by = {}
    for (disp, c), v in per.items():
        by.setdefault(c, {})[disp] = v
    return by


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pmc-dir", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--units-per-dispatch", type=float, required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--sources", choices=["fast", "act"], required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--commit", default="unknown")
    ap.add_argument("--kernel-us", type=float, default=0.0, help="measured mean dispatch duration (effective clock)")
    a = ap.parse_args()
    import bench
    by = counters(a.pmc_dir, a.kernel)
    if "SQ_INSTS_VALU" not in by:
        sys.exit(f"no SQ_INSTS_VALU rows for /{a.kernel}/ under {a.pmc_dir}")
    n = len(by["SQ_INSTS_VALU"])
    mean = lambda c: sum(by[c].values()) / len(by[c]) if c in by and by[c] else None
    valu = mean("SQ_INSTS_VALU")
    grbm = mean("GRBM_GUI_ACTIVE")
    rec = {"valu_lane_instr_per_unit": round(valu * 64 / a.units_per_dispatch, 4),
           "valu_insts_per_dispatch": valu, "units_per_dispatch": a.units_per_dispatch, "dispatches": n,
           "kernel_regex": a.kernel, "commit": a.commit, "date": datetime.date.today().isoformat(),
           "kernel_source_sha256": bench.kernel_source_hash(bench.KERNEL_SOURCES if a.sources == "fast"
                                                            else bench.ACT_SOURCES)}
    act, act2 = mean("SQ_ACTIVE_INST_VALU"), mean("SQ_ACTIVE_INST_VALU2")
    if act is not None and act2 is not None:
        rec["valu_slots_per_unit"] = round((act - act2) / a.units_per_dispatch, 6)
        rec["dual_issued_instr_frac"] = round(2 * act2 / valu, 4)
    if grbm:
        cycles = grbm / 8
        rec["dispatch_cycles"] = cycles
        if act is not None and act2 is not None:
            rec["valu_slot_occupancy"] = round((act - act2) / (cycles / 4 * 1024), 4)
        if a.kernel_us:
            rec["effective_clock_ghz"] = round(cycles / (a.kernel_us * 1e3), 3)
    for c in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_SALU", "SQ_WAIT_INST_ANY",
              "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VALU2"):
        if c in by:
            rec[c] = mean(c)
    try:
        with open(a.out) as f:
            allrec = json.load(f)
    except (OSError, ValueError):
        allrec = {}
    allrec[a.key] = rec
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(allrec, f, indent=1, sort_keys=True)
    print(json.dumps({a.key: rec}))


if __name__ == "__main__":
    main()
