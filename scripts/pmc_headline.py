#!/usr/bin/env python3
"""Per-wave view of the headline kernel vs its memory-structure ceiling from the
pmc_headline.sh summaries: cycles a wave lives, how many of them it waits (any wait /
waiting for an instruction's dependency), issues, and the HBM bytes per launch.

SQ_* cycle counters are quad-cycles summed over the SEs that report them; ratios between
counters of one kernel are what this prints, plus per-wave means (value / SQ_WAVES)."""
import json
import os
import sys

d = sys.argv[1]
summ = {}
for name in ("sq_a", "sq_b", "fetch", "write"):
    p = os.path.join(d, f"{name}.summary.json")
    if os.path.exists(p):
        with open(p) as f:
            for k, cs in json.load(f).items():
                short = "awq_fast_kernel" if "awq_fast_kernel" in k else ("ceiling" if "ceiling" in k else k[:40])
                for c, v in cs.items():
                    summ.setdefault(short, {})[c] = v["median"]
out = {}
for k, c in summ.items():
    waves = c.get("SQ_WAVES") or 1
    r = {"waves": waves}
    for n in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
              "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS",
              "SQ_ACTIVE_INST_SCA", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS"):
        if n in c:
            r[n + "_per_wave"] = round(c[n] / waves, 2)
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in c:
                r[n + "_over_wave_cycles"] = round(c[n] / wc, 4)
    if "FETCH_SIZE" in c:
        r["hbm_read_bytes (bytes = FETCH_SIZE KiB x 1024 x 2, gfx950 half-count)"] = c["FETCH_SIZE"] * 2048
    if "WRITE_SIZE" in c:
        r["hbm_write_bytes (bytes = WRITE_SIZE KiB x 1024)"] = c["WRITE_SIZE"] * 1024
    if "GRBM_GUI_ACTIVE" in c:
        r["GRBM_GUI_ACTIVE"] = c["GRBM_GUI_ACTIVE"]
    out[k] = r
print(json.dumps(out, indent=1))
