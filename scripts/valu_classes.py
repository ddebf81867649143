#!/usr/bin/env python3
"""Per-instruction-class VALU issue table of gfx950 from scripts/valu_probe: the probe's own
timing (cycles per instruction per SIMD at 8 waves per SIMD) joined with two rocprofv3 --pmc
passes over the same binary (A: SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_ACTIVE_INST_VALU2,
per-type counts; B: more per-type counts).  What it shows (profiles/round5/r5k/):

  * SQ_ACTIVE_INST_VALU counts one quad-cycle per VALU instruction (two for v_exp / v_rcp);
  * SQ_ACTIVE_INST_VALU2 counts the quad-cycles in which a SIMD issued two VALU instructions:
    only plain f32 add / sub / mul / fma, f16 mul, v_mov_b32, v_and_b32, v_add_u32 pair
    (~2.4-2.7 cycles each); conversions, v_rndne, v_med3 / v_max / v_min, DPP, packed f32 /
    f16, v_fma_mix, shifts and 3-operand integer ops take a quad-cycle each (~4.1-4.7);
  * so the issue slots a kernel occupies are SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2, one
    slot per SIMD per quad-cycle — the VALU roofline bench.py --mode search / act uses.

  valu_classes.py --probe-log DIR/probe.log --pmc-a DIR/probe_a --pmc-b DIR/probe_b [--out J]
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(d):
    per = collections.defaultdict(float)
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                per[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"] or 0)
    by = collections.defaultdict(dict)
    for (d_, c), v in per.items():
        by[d_][c] = v
    return by


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--probe-log", required=True)
    ap.add_argument("--pmc-a", required=True)
    ap.add_argument("--pmc-b", required=True)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    with open(a.probe_log) as f:
        runs = [json.loads(line) for line in f if line.startswith('{"op"')]
    ops = [r["op"] for r in runs if r["waves_per_simd"] == 8]
    cyc = {r["op"]: r["cycles_per_instr_per_simd"] for r in runs if r["waves_per_simd"] == 8}
    A, B = load(a.pmc_a), load(a.pmc_b)
    da, db = sorted(A), sorted(B)
    per_op = 4   # warm-up + timed launch at 2 and at 8 waves per SIMD
    if len(da) != per_op * len(ops) or len(db) != per_op * len(ops):
        raise SystemExit(f"expected {per_op * len(ops)} dispatches, got {len(da)} / {len(db)}")
    table = []
    for i, op in enumerate(ops):
        ca, cb = A[da[per_op * i + 3]], B[db[per_op * i + 3]]   # the timed 8-wave launch
        n = ca["SQ_INSTS_VALU"]
        quads = ca["GRBM_GUI_ACTIVE"] / 8 / 4 * 1024           # quad-cycles x SIMDs
        types = {k.replace("SQ_INSTS_VALU_", ""): round(v / n, 3) for k, v in {**ca, **cb}.items()
                 if k.startswith("SQ_INSTS_VALU_") and v / n > 0.01}
        table.append({"op": op, "cycles_per_instr": cyc[op],
                      "active_quads_per_instr": round(ca["SQ_ACTIVE_INST_VALU"] / n, 3),
                      "dual_issue_quads_per_instr": round(ca["SQ_ACTIVE_INST_VALU2"] / n, 3),
                      "slot_occupancy": round((ca["SQ_ACTIVE_INST_VALU"] - ca["SQ_ACTIVE_INST_VALU2"]) / quads, 3),
                      "type_counters": types})
    text = json.dumps(table, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    for t in table:
        print(f'{t["op"]:20s} {t["cycles_per_instr"]:6.2f} cyc  active {t["active_quads_per_instr"]:.2f}  '
              f'dual {t["dual_issue_quads_per_instr"]:.2f}  slots busy {t["slot_occupancy"]:.2f}  {t["type_counters"]}')


if __name__ == "__main__":
    main()
