#!/usr/bin/env python3
"""Algorithmic VALU floor of the two grid searches, and where each kernel's
issue slots above that floor go.

FLOOR: the per-candidate-element instruction chain the reference's per-op rounding forces
(awq.py:245-248 quantize, awq.py:459-539 dequantize; every bf16 / fp16 rounding is a
conversion on gfx950), each step priced with the cheapest exact gfx950 instruction and the
issue-slot model of profiles/round5/r5k/valu_classes.json: a dual-issue-class
instruction (plain f32 add / sub / mul / fma, v_and / v_mov / v_add_u32) costs 1/2 slot, a packed
f32 instruction (v_pk_add/mul_f32: two elements) 1 slot = 1/2 per element, conversions /
v_rndne / v_med3 / v_max / v_min / v_fma_mix / shifts 1 slot (v_cvt_pk_*: two elements per slot).
Per-group work (the candidate's parameters, broadcasts, the error tree across lanes) is NOT in
the floor: it is amortised over the group (128 elements) and is what the gap names.

GAP: the kernel's hot loop in the ISA (`make -C awq-converter_amd/csrc isa ISA_SRC=awq_fast` /
`ISA_SRC=awq_actsearch`), its VALU instructions per element priced the same way and grouped by
what they do, beside the measured slots per unit (profiles/round6/pmc_valu.json) and the
per-type VALU counters of the same commands (profiles/round6/r6fk/{search,act}_{a,b}).

  python scripts/valu_floor.py [--write profiles/round6/valu_floor.json]
"""
import argparse
import collections
import json
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "awq-converter_amd", "csrc")

# (step, instruction, slots per element, instructions per element, PMC type counter the
# instruction increments: CVT / ADD_F32 / MUL_F32 / FMA_F32 / OTHER = none of the per-type
# counters: v_rndne, v_med3, v_min/max, DPP, compares, selects, moves, bit ops)
# bf16 rounding kept in f32 form: v_cvt_pk_bf16_f32 with a zero low half writes RN_bf16(v) as
# the f32 it is (1 slot per element; two elements per conversion would need a 1.5-slot unpack).
FLOOR = {
    # clip search, bf16 weights, asymmetric 4-bit (bench --mode search's line): per candidate and element
    "search.bf16.asym": [
        ("RN(x * r): product", "v_pk_mul_f32 (2 elements)", 0.5, 0.5, "MUL_F32"),
        ("RN(x * r): round to bf16", "v_cvt_pk_bf16_f32 (zero low half)", 1.0, 1.0, "CVT"),
        ("+ z", "v_pk_add_f32", 0.5, 0.5, "ADD_F32"),
        ("RN to bf16", "v_cvt_pk_bf16_f32 (zero low half)", 1.0, 1.0, "CVT"),
        # (round 6: the integer steps in packed fp16, two elements per instruction — cheaper than
        #  v_rndne + v_med3 + f32 (q - z) * s + v_cvt_pk_f16; exhaustive: verify_recip chain16)
        ("u to fp16 (exact where it matters)", "v_cvt_pk_f16_f32 (2 elements)", 0.5, 0.5, "CVT"),
        ("rint (half even): + (1024 - qmin)", "v_pk_add_f16", 0.5, 0.5, "ADD_F16"),
        ("clamp(1024, 1024 + qmax - qmin)", "v_pk_max_f16 + v_pk_min_f16", 1.0, 1.0, "OTHER"),
        ("q - z (exact)", "v_pk_add_f16", 0.5, 0.5, "ADD_F16"),
        ("(q - z) * fp16 scale (the reference's fp16 product)", "v_pk_mul_f16", 0.5, 0.5, "MUL_F16"),
        ("x - dq (fp16 operand)", "v_fma_mix_f32", 1.0, 1.0, "FMA_F32"),
        ("square", "v_pk_mul_f32", 0.5, 0.5, "MUL_F32"),
        ("ordered add (two chunk accumulators per packed add)", "v_pk_add_f32", 0.5, 0.5, "ADD_F32"),
    ],
    # activation-aware loss, bf16 weights, asymmetric 4-bit (bench --mode act's line)
    "act.bf16.asym": [
        ("w' = RN(w * s_k): product", "v_pk_mul_f32", 0.5, 0.5, "MUL_F32"),
        ("w': round to bf16", "v_cvt_pk_bf16_f32 (zero low half)", 1.0, 1.0, "CVT"),
        ("group min / max of w' (two new elements per 3-operand op)", "v_min3_f32 + v_max3_f32", 1.0, 1.0, "OTHER"),
        ("RN(w' * r): product", "v_pk_mul_f32", 0.5, 0.5, "MUL_F32"),
        ("RN to bf16", "v_cvt_pk_bf16_f32 (zero low half)", 1.0, 1.0, "CVT"),
        ("+ z", "v_pk_add_f32", 0.5, 0.5, "ADD_F32"),
        ("RN to bf16", "v_cvt_pk_bf16_f32 (zero low half)", 1.0, 1.0, "CVT"),
        ("u to fp16 (exact where it matters)", "v_cvt_pk_f16_f32 (2 elements)", 0.5, 0.5, "CVT"),
        ("rint (half even): + (1024 - qmin)", "v_pk_add_f16", 0.5, 0.5, "ADD_F16"),
        ("clamp(1024, 1024 + qmax - qmin)", "v_pk_max_f16 + v_pk_min_f16", 1.0, 1.0, "OTHER"),
        ("q - z (exact)", "v_pk_add_f16", 0.5, 0.5, "ADD_F16"),
        ("(q - z) * fp16 scale", "v_pk_mul_f16", 0.5, 0.5, "MUL_F16"),
        ("dq / s_k: q0 = dq * rs (fp16 operand)", "v_fma_mix_f32", 1.0, 1.0, "FMA_F32"),
        ("dq / s_k: r = fma(-s, q0, dq) (fp16 operand)", "v_fma_mix_f32", 1.0, 1.0, "FMA_F32"),
        ("dq / s_k: fma(r, rs, q0)", "v_pk_fma_f32", 0.5, 0.5, "FMA_F32"),
        ("e = w_hat - w", "v_pk_add_f32", 0.5, 0.5, "ADD_F32"),
        ("x_sq * (e * e)", "2 x v_pk_mul_f32", 1.0, 1.0, "MUL_F32"),
        ("ordered add", "v_pk_add_f32", 0.5, 0.5, "ADD_F32"),
    ],
}

# the per-type counter passes of the same bench commands (scripts/cmd/r6fk.sh; the A / B counter sets
# of scripts/valu_classes.py): dynamic instructions per type for the kernel's launches
TYPE_PASSES = {"search.bf16.asym": ("search_a", "search_b", "awq_fast_kernel"),
               "act.bf16.asym": ("act_a", "act_b", "act_loss_kernel")}


def dynamic_types(r5k, key, lane_instr_per_unit):
    """Lane instructions per unit by PMC type (SQ_INSTS_VALU_*), scaled so they sum to the
    recorded lane instructions per unit; OTHER = the VALU instructions no type counter counts."""
    import csv
    import glob
    a, b, kern = TYPE_PASSES[key]
    tot = collections.defaultdict(float)
    for d in (a, b):
        for p in glob.glob(os.path.join(r5k, d, "**", "*counter_collection.csv"), recursive=True):
            with open(p) as f:
                for r in csv.DictReader(f):
                    if kern in r["Kernel_Name"]:
                        tot[(d, r["Counter_Name"])] += float(r["Counter_Value"] or 0)
    n = tot.get((a, "SQ_INSTS_VALU"))
    if not n:
        return None
    per = {}
    for (d, c), v in tot.items():
        if c.startswith("SQ_INSTS_VALU_") and v:
            per[c.replace("SQ_INSTS_VALU_", "")] = v / n * lane_instr_per_unit
    per["OTHER"] = lane_instr_per_unit - sum(per.values())
    return {k: round(v, 3) for k, v in sorted(per.items(), key=lambda kv: -kv[1])}


DUAL = re.compile(r"v_(add|sub|subrev|mul|fma|fmac|mac)_f32_e32$|v_(add|sub|subrev|mul|fma|fmac)_f32$|"
                  r"v_fma_f32$|v_mov_b32_e32$|v_and_b32_e32$|v_add_u32_e32$|v_mul_f16_e32$")

CATEGORY = [   # (name, regex on the opcode) — first match wins
    ("dpp reductions / broadcasts", r".*_dpp$|v_permlane.*|v_readlane.*|v_readfirstlane.*"),
    ("fp16 -> f32 widening", r"v_cvt_f32_f16.*"),
    ("bf16 / fp16 rounding", r"v_cvt_pk_(bf16|f16)_f32|v_cvt_f16_f32.*|v_cvt_pk_u8.*"),
    ("rint / clamp", r"v_rndne.*|v_med3.*"),
    ("min / max", r"v_(min|max)(3)?_f32.*"),
    ("packed f32 arithmetic", r"v_pk_(add|mul|fma)_f32"),
    ("packed fp16 arithmetic (rint by + 1024, clamp, q - z, * s)", r"v_pk_(add|mul|fma|max|min|sub)_f16"),
    ("f32 add / sub / mul / fma", r"v_(add|sub|subrev|mul|fma|fmac)_f32.*|v_fma_mix.*"),
    ("candidate parameters (division, reciprocal)", r"v_div_.*|v_rcp.*|v_frexp.*|v_ldexp.*"),
    ("compares / selects", r"v_cmp.*|v_cndmask.*"),
    ("integer / bit ops, moves", r"v_.*"),
]


def slots(op: str) -> float:
    if op.startswith("v_pk_"):
        return 1.0
    if DUAL.match(op):
        return 0.5
    if op.startswith(("v_rcp", "v_exp", "v_log", "v_sqrt", "v_rsq")):
        return 2.0
    return 1.0


def function_body(asm: str, name_rx: str):
    m = re.search(r"^(" + name_rx + r"):", asm, re.M)
    if not m:
        raise SystemExit(f"no function matching {name_rx}")
    i = m.start()
    return m.group(1), asm[i:asm.index(".Lfunc_end", i)].split("\n")


def hot_loop(body, rint_per_iter):
    """The smallest backward-branch region holding exactly `rint_per_iter` v_rndne (one per
    element of a candidate): the candidate loop's common path."""
    labels = {}
    for n, line in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", line.strip())
        if m:
            labels[m.group(1)] = n
    best = None
    for n, line in enumerate(body):
        m = re.match(r"\s*s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", line)
        if m and m.group(1) in labels and labels[m.group(1)] < n:
            a = labels[m.group(1)]
            ops = [x.strip().split()[0] for x in body[a:n + 1]
                   if x.strip() and not x.strip().startswith((";", ".")) and x.strip().split()[0].startswith("v_")]
            if rint_per_iter <= sum(o.startswith("v_rndne") for o in ops) <= rint_per_iter + 2 and \
                    (best is None or len(ops) < len(best[2])):
                best = (a, n, ops)
    return best


def common_path_loop(body, rint_per_iter, marker="v_rndne"):
    """The candidate loop's common path: over the blocks of an inner loop (the compiler's
    "in Loop: Header=" block comments), the cheapest path in VALU slots from the header back to
    it — the rare branches (IEEE divisions for n_grid > 65536, 0 / inf / NaN scales, fp16 scales
    >= 14) are the longer ones.  Returns (header line, VALU opcodes) for the first inner-loop
    header whose cheapest iteration holds `rint_per_iter` .. + 2 `marker` instructions (one per
    element and candidate: KERNELS), or None (hot_loop is the fallback)."""
    starts, names = [], []
    for n, line in enumerate(body):
        s = line.strip()
        m = re.match(r"^(\.LBB\w+):", s) or re.match(r"^; (%bb\.\d+):", s)
        if m:
            starts.append(n)
            names.append(m.group(1))
    idx = {nm: i for i, nm in enumerate(names)}
    ends = starts[1:] + [len(body)]

    def instrs(i):
        return [x.strip() for x in body[starts[i] + 1:ends[i]]
                if x.strip() and not x.strip().startswith((";", "."))]

    def comment(i):
        return " ".join(body[k] for k in range(starts[i], min(starts[i] + 3, len(body))))

    for h in range(len(starts)):
        if "Inner Loop Header" not in comment(h):
            continue
        hname = names[h].lstrip(".L")
        member = {i for i in range(len(starts)) if f"Header={hname} " in comment(i) or i == h}
        memo = {}

        def best(i, need, depth=0):
            """(slots, ops) of the cheapest path from block i to the back edge holding exactly
            `need` marker instructions"""
            key = (i, need)
            if key in memo:
                return memo[key]
            memo[key] = (float("inf"), [])          # cycle guard
            ins = instrs(i)
            ops = [x.split()[0] for x in ins if x.split()[0].startswith("v_")]
            left = need - sum(o.startswith(marker) for o in ops)
            if left < 0:
                return memo[key]
            last = ins[-1].split() if ins else [""]
            if last[0] == "s_branch":
                succ = [idx.get(last[1], -1)]
            elif last[0].startswith("s_cbranch_"):
                succ = [i + 1, idx.get(last[1], -1)]
            else:
                succ = [i + 1]
            cands = []
            for j in succ:
                if j == h:
                    cands.append((0.0, []) if left == 0 else (float("inf"), []))
                elif j in member and depth < 300:
                    cands.append(best(j, left, depth + 1))
            c, o = min(cands, key=lambda t: t[0]) if cands else (float("inf"), [])
            memo[key] = (c + sum(slots(x) for x in ops), ops + o)
            return memo[key]

        for need in range(rint_per_iter, rint_per_iter + 3):
            cost, ops = best(h, need)
            if cost < float("inf"):
                return starts[h], ops
    return None


def categorize(ops, elements):
    out = collections.OrderedDict((c, 0.0) for c, _ in CATEGORY)
    for o in ops:
        for c, rx in CATEGORY:
            if re.fullmatch(rx, o):
                out[c] += slots(o) / elements
                break
    return {k: round(v, 3) for k, v in out.items() if v}


KERNELS = {
    "search.bf16.asym": dict(src="awq_fast", fn=r"_ZN3awq12_GLOBAL__N_115awq_fast_kernelINS0_7FmtBF16ELi4ELb0ELb1ELi128ELb0ELb0EE\w*",
                             elements=32, marker="v_fma_mix_f32", pmc_key="llama3-8b.b4.asym.packed.search10of20"),
    "act.bf16.asym": dict(src="awq_actsearch", fn=r"_ZN3awq12_GLOBAL__N_115act_loss_kernelILi0ELi8ELb0ELi16EE\w*",
                          elements=16, marker="v_fma_mix_f32", markers_per_element=2,
                          pmc_key="act.llama3-8b-block.t512.g20.bf16.b4.asym"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "round6", "pmc_valu.json"))
    ap.add_argument("--types-dir", default="search=" + os.path.join(ROOT, "profiles", "round6", "r6fk") + ",act="
                    + os.path.join(ROOT, "profiles", "round6", "r6fk"),
                    help="kind=dir,...: the per-type counter passes (search_a/b, act_a/b: scripts/cmd/r6fk.sh, "
                         "the final tree)")
    ap.add_argument("--write", default="")
    ap.add_argument("--no-isa", action="store_true", help="floors only (no hipcc)")
    a = ap.parse_args()
    pmc = json.load(open(a.pmc))
    out = {}
    for key, chain in FLOOR.items():
        fl = sum(c[2] for c in chain)
        k = KERNELS[key]
        rec = pmc.get(k["pmc_key"], {})
        meas = rec.get("valu_slots_per_unit")
        floor_types = collections.defaultdict(float)
        for c in chain:
            floor_types[c[4]] += c[3]
        r = {"floor_slots_per_element": fl, "floor_slots_per_unit": round(fl / 64, 6),
             "floor_instructions_per_element": sum(c[3] for c in chain),
             "floor_instructions_by_type": dict(floor_types),
             "chain": [{"step": c[0], "instruction": c[1], "slots": c[2]} for c in chain],
             "measured_slots_per_unit": meas, "measured_source": f"{os.path.relpath(a.pmc, ROOT)}:{k['pmc_key']}",
             "unit": "candidate-element (one element scored for one candidate); slots per unit = slots per element / 64"}
        if meas:
            r["measured_over_floor"] = round(meas / (fl / 64), 3)
            r["measured_slots_per_element"] = round(meas * 64, 3)
        lane = rec.get("valu_lane_instr_per_unit")
        if lane:
            tdirs = dict(kv.split("=", 1) for kv in a.types_dir.split(","))
            tdir = tdirs[key.split(".")[0]]
            dyn = dynamic_types(tdir, key, lane)
            r["types_source"] = os.path.relpath(tdir, ROOT)
            if dyn:
                r["measured_instructions_by_type"] = dyn
                r["excess_instructions_by_type"] = {t: round(v - floor_types.get(t, 0.0), 3) for t, v in dyn.items()}
        if not a.no_isa:
            sfile = os.path.join(CSRC, "build", f"{k['src']}-hip-amdgcn-amd-amdhsa-gfx950.s")
            if not os.path.exists(sfile):
                subprocess.run(["make", "-s", "-C", CSRC, "isa", f"ISA_SRC={k['src']}"], check=True)
            name, body = function_body(open(sfile).read(), k["fn"])
            walk = common_path_loop(body, k["elements"] * k.get("markers_per_element", 1), k.get("marker", "v_rndne"))
            loop = (walk[0], None, walk[1]) if walk else hot_loop(body, k["elements"])
            if loop:
                a0, a1, ops = loop
                cats = categorize(ops, k["elements"])
                r["isa"] = {"function": name, "loop_lines": [a0, a1], "valu_instructions": len(ops),
                            "loop_extraction": "common-path walk from the loop header" if walk
                            else "smallest backward-branch region",
                            "elements_per_iteration": k["elements"],
                            "loop_slots_per_element": round(sum(slots(o) for o in ops) / k["elements"], 3),
                            "loop_slots_per_element_by_category": cats,
                            "opcodes": dict(collections.Counter(ops).most_common())}
        out[key] = r
        print(json.dumps({key: {x: r[x] for x in ("floor_slots_per_element", "floor_slots_per_unit",
                                                  "measured_slots_per_unit", "measured_over_floor",
                                                  "excess_instructions_by_type") if x in r}}))
        if "isa" in r:
            print("   loop slots/element", r["isa"]["loop_slots_per_element"], r["isa"]["loop_slots_per_element_by_category"])
    if a.write:
        with open(a.write, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
