#!/usr/bin/env python3
"""Generate the golden fixtures that pin the oracle (and through it the HIP path).

TEST INFRASTRUCTURE ONLY — this script imports the *reference* implementation
(shanefitch/AWQ-Converter, mounted read-only at /root/reference) in THIS
container, runs ``AWQQuantizer.quantize()`` / ``dequantize()`` /
``quantize_model()`` on CPU, and writes inputs + outputs as data files:

  tests/golden/golden_small.safetensors   inputs and full outputs of small cases
  tests/golden/golden_manifest.json       per-case parameters, SHA-256 digests of
                                          large cases, error/behaviour records

Nothing from the reference is copied: only the numbers it produced.  The
reference is never imported by tests, bench.py or the product; the GPU box
never sees /root/reference.  Re-run with:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --nan   (golden_nan.*)

Reference call sites pinned here:
  awq.py:376-433  quantize()            awq.py:459-539 dequantize()
  awq.py:435-457  quantize_model()      awq.py:95-112  _validate_parameters()
  awq.py:286-374  _quantize_per_group() awq.py:130-171 _calculate_scale_zp()
"""
import hashlib
import json
import logging
import os
import sys

REF_SRC = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))

if not os.path.isdir(REF_SRC):
    sys.exit("make_golden.py: /root/reference is absent — fixtures can only be "
             "generated in the build container (the GPU box uses the committed files)")

sys.dont_write_bytecode = True
sys.path.insert(0, REF_SRC)

import torch  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

from awq_quantizer.quantization.awq import AWQQuantizer  # noqa: E402  (reference)

logging.disable(logging.CRITICAL)
torch.set_num_threads(8)

DTYPES = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32, "f64": torch.float64}


def sha(t: torch.Tensor) -> str:
    t = t.contiguous()
    if t.dtype == torch.bfloat16:
        t = t.view(torch.int16)
    return hashlib.sha256(t.numpy().tobytes()).hexdigest()


def rand_input(shape, seed, dtype, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g, dtype=torch.float32) * scale).to(dtype)


def edge_rows_f32():
    """16 rows x 256 (2 groups at gs=128) of hand-built edge cases (float32, cast per dtype)."""
    K = 256
    rows = []
    g = torch.Generator().manual_seed(1234)
    r = lambda: torch.randn(K, generator=g)
    rows.append(torch.zeros(K))                                   # 0 all-zero
    rows.append(torch.full((K,), 1e-6))                           # 1 constant tiny
    rows.append(1.0 + torch.rand(K, generator=g))                 # 2 all-positive
    rows.append(-1.0 - torch.rand(K, generator=g))                # 3 all-negative
    x = r(); x[5] = float("nan"); rows.append(x)                  # 4 NaN in group 0
    x = r(); x[3] = float("inf"); x[200] = float("-inf"); rows.append(x)  # 5 +inf g0, -inf g1
    x = torch.full((K,), 5.0); x[7] = float("inf"); x[9] = float("-inf"); rows.append(x)  # 6 ±inf g0
    x = (torch.arange(K) % 31).float() * 0.5; rows.append(x)      # 7 half-steps 0..15 -> ties
    x = r().sign() * 1e38; x[0] = 3.0e38; rows.append(x)          # 8 huge magnitude
    x = r() * 1e-39; rows.append(x)                               # 9 subnormal (f32/bf16)
    x = torch.zeros(K); x[1::2] = -0.0; x[150] = 0.75; rows.append(x)  # 10 signed zeros
    x = torch.linspace(-1.25, 6.25, K); rows.append(x)            # 11 zero-point tie (-2.5 -> 2)
    x = torch.zeros(K); x[0] = 3e38; x[1] = -3e38; x[128] = 2e38; x[129] = -2e38; rows.append(x)  # 12 overflow spread
    x = 1.0 + torch.rand(K, generator=g) * 0.0078125; rows.append(x)  # 13 narrow range, large offset
    rows.append(r() * 1e-4)                                       # 14 small random
    rows.append(r() * 100.0)                                      # 15 large random
    return torch.stack(rows)


def run_case(params, x):
    q = AWQQuantizer(device="cpu", **params)
    out = {"ok": True}
    try:
        res = q.quantize(x)
    except Exception as e:  # record behaviour, e.g. percentile TypeError
        return {"ok": False, "error": type(e).__name__, "message": str(e)}, None
    try:
        dq = q.dequantize(res)
        out["dequantize"] = "ok"
    except Exception as e:
        dq = None
        out["dequantize"] = type(e).__name__
    return out, (res, dq)


def main():
    tensors = {}
    manifest = {"generator": "tests/golden/make_golden.py", "torch": torch.__version__,
                "reference": "shanefitch/AWQ-Converter src/awq_quantizer/quantization/awq.py",
                "cases": [], "hashed": [], "validation": [], "quantize_model": {}}

    # ---- small cases: full inputs + outputs stored ----
    small = []
    edge = edge_rows_f32()
    for dn in ("bf16", "f16", "f32", "f64"):
        dt = DTYPES[dn]
        shapes = [("edge", edge.to(dt)),
                  ("r8x300", rand_input((8, 300), 11, dt)),
                  ("pos8x300", rand_input((8, 300), 12, dt).abs() + 0.5),
                  ("neg8x300", -(rand_input((8, 300), 13, dt).abs() + 0.5)),
                  ("v1000", rand_input((1000,), 14, dt, 0.02)),
                  ("v768", rand_input((768,), 15, dt)),
                  ("t4x3x100", rand_input((4, 3, 100), 16, dt)),
                  ("r16x512", rand_input((16, 512), 17, dt, 0.02)),
                  ("s10x10", rand_input((10, 10), 18, dt)),
                  ("s100", rand_input((100,), 19, dt)),
                  ("s0d", torch.tensor(1.5, dtype=dt)),
                  ("s3x5x7", rand_input((3, 5, 7), 20, dt))]
        for sn, x in shapes:
            for sym in (False, True):
                for bits in (4, 8):
                    gss = [128]
                    if sn in ("r8x300", "r16x512", "t4x3x100") and bits == 4:
                        gss = [128, 64, 32, 100, 256]
                    pcs = [True, False] if sn.startswith("s") else [True]
                    for gs in gss:
                        for pc in pcs:
                            small.append((f"{dn}.{sn}.{'sym' if sym else 'asym'}.b{bits}.g{gs}.pc{int(pc)}",
                                          dict(bits=bits, group_size=gs, symmetric=sym, per_channel=pc), x,
                                          f"in.{dn}.{sn}"))
    for name, params, x, in_key in small:
        rec, res = run_case(params, x)
        rec.update(name=name, params=params, shape=list(x.shape), dtype=str(x.dtype), input=in_key)
        manifest["cases"].append(rec)
        key = name
        if in_key not in tensors:
            xs = x.view(torch.int16) if x.dtype == torch.bfloat16 else x
            tensors[in_key] = xs.contiguous().clone()
        if res is not None:
            r, dq = res
            tensors[key + ".tensor_q"] = r["tensor_q"].contiguous()
            tensors[key + ".scales"] = r["scales"].contiguous()
            tensors[key + ".zero_points"] = r["zero_points"].contiguous()
            for k in ("bits", "group_size", "symmetric"):
                rec[k] = r[k].item()
            rec["out_shapes"] = {k: list(r[k].shape) for k in ("tensor_q", "scales", "zero_points")}
            if dq is not None and params["group_size"] == 128:   # keep the fixture small
                tensors[key + ".dq"] = dq.contiguous()
        print(name, rec.get("ok"), rec.get("dequantize", rec.get("error")), flush=True)

    # percentile mode (always raises inside the reference, awq.py:189 -> tensor_utils.py:87)
    x = rand_input((4, 256), 21, torch.bfloat16)
    rec, _ = run_case(dict(bits=4, group_size=128, symmetric=False, zero_point="percentile"), x)
    rec.update(name="bf16.percentile")
    manifest["cases"].append(rec)
    # zero_point="none" behaves like minmax (only "percentile" is special, awq.py:187)
    rec, res = run_case(dict(bits=4, group_size=128, symmetric=False, zero_point="none"), x)
    rec.update(name="bf16.zp_none.asym.b4.g128", params=dict(bits=4, group_size=128, symmetric=False,
                                                              zero_point="none"), shape=[4, 256], dtype=str(x.dtype),
               input="in.bf16.zp_none")
    tensors["in.bf16.zp_none"] = x.view(torch.int16).clone()
    tensors[rec["name"] + ".tensor_q"] = res[0]["tensor_q"]
    tensors[rec["name"] + ".scales"] = res[0]["scales"]
    tensors[rec["name"] + ".zero_points"] = res[0]["zero_points"]
    manifest["cases"].append(rec)

    # ---- large cases: seeded inputs, SHA-256 of outputs ----
    big = [("bf16", (1024, 4096), 0, 1.0, False, 4), ("bf16", (1024, 4096), 0, 1.0, True, 4),
           ("bf16", (1024, 4096), 0, 1.0, False, 8), ("bf16", (1024, 4096), 0, 1.0, True, 8),
           ("bf16", (768, 3072), 1, 1.0, False, 4), ("bf16", (768, 3, 768), 2, 1.0, False, 4),
           ("bf16", (512, 4096), 3, 0.02, False, 4), ("f16", (1024, 4096), 0, 1.0, False, 4),
           ("f16", (512, 4096), 3, 0.02, True, 4), ("f32", (256, 4096), 4, 1.0, False, 4)]
    for dn, shape, seed, scale, sym, bits in big:
        x = rand_input(shape, seed, DTYPES[dn], scale)
        params = dict(bits=bits, group_size=128, symmetric=sym, per_channel=True)
        rec, res = run_case(params, x)
        r, dq = res
        rec.update(name=f"{dn}.{'x'.join(map(str, shape))}.seed{seed}.sc{scale}.{'sym' if sym else 'asym'}.b{bits}",
                   params=params, shape=list(shape), dtype=dn, seed=seed, scale=scale,
                   sha_x=sha(x), sha_tensor_q=sha(r["tensor_q"]), sha_scales=sha(r["scales"]),
                   sha_zero_points=sha(r["zero_points"]), sha_dq=sha(dq) if dq is not None else None)
        manifest["hashed"].append(rec)
        print(rec["name"], flush=True)

    # ---- parameter validation messages (awq.py:95-112) ----
    bad = [dict(bits=3), dict(bits=16), dict(group_size=0), dict(group_size=-4),
           dict(zero_point="foo"), dict(zero_point="percentile", percentile=0.0),
           dict(zero_point="percentile", percentile=1.0), dict(scale_method="bar")]
    for p in bad:
        try:
            AWQQuantizer(device="cpu", **p)
            manifest["validation"].append({"params": p, "error": None})
        except Exception as e:
            manifest["validation"].append({"params": p, "error": type(e).__name__, "message": str(e)})
    q = AWQQuantizer(device="cpu")
    for label, arg in (("list", [1.0, 2.0]), ("int", torch.arange(256, dtype=torch.int32))):
        try:
            q.quantize(arg)
        except Exception as e:
            manifest["validation"].append({"quantize_arg": label, "error": type(e).__name__, "message": str(e)})

    # ---- quantize_model skip semantics (awq.py:435-457) ----
    model = {"w": rand_input((8, 256), 30, torch.bfloat16), "i": torch.arange(256, dtype=torch.int32),
             "s": rand_input((10, 10), 31, torch.bfloat16), "e": torch.zeros(0, dtype=torch.bfloat16),
             "b": rand_input((256,), 32, torch.bfloat16)}
    out = AWQQuantizer(device="cpu", symmetric=False).quantize_model(model)
    manifest["quantize_model"]["asym"] = sorted(out.keys())
    out = AWQQuantizer(device="cpu", zero_point="percentile").quantize_model(model)
    manifest["quantize_model"]["percentile"] = sorted(out.keys())

    save_file(tensors, os.path.join(HERE, "golden_small.safetensors"))
    with open(os.path.join(HERE, "golden_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("cases", len(manifest["cases"]), "hashed", len(manifest["hashed"]),
          "bytes", os.path.getsize(os.path.join(HERE, "golden_small.safetensors")))


# ---------------------------------------------------------------- NaN-origin cases (--nan)
# The fp16 bits of a NaN scale depend on where the NaN came from and on the input dtype
# (awq.py:192-205 reductions and arithmetic, the fp32 scale buffer of awq.py:327/352, the
# .to(float16) of awq.py:411).  These cases pin that: +NaN / -NaN / payload / signalling
# NaNs, NaN next to +-inf, all-inf groups (inf - inf), NaN in a zero-padded tail group,
# group sizes 1 / 2 / 3, scale tensors of 1, 7, 8, 9, 16, 17, 33 and 51 elements, and the
# small-tensor path (awq.py:130-171: whole tensor and per row, one element and more).
# Written to golden_nan.safetensors / golden_nan.json.

_IT = {torch.bfloat16: torch.int16, torch.float16: torch.int16, torch.float32: torch.int32,
       torch.float64: torch.int64}


def nan_bits(dt, kind):
    """A NaN of dtype dt as a 0-d tensor: 'p' +qNaN, 'n' -qNaN, 'pay' qNaN with a payload,
    's' signalling NaN (payload 1), 'nspay' negative signalling NaN with payload 3."""
    w = {torch.bfloat16: 16, torch.float16: 16, torch.float32: 32, torch.float64: 64}[dt]
    e = {torch.bfloat16: 8, torch.float16: 5, torch.float32: 8, torch.float64: 11}[dt]
    m = w - 1 - e
    exp = ((1 << e) - 1) << m
    q = 1 << (m - 1)
    v = {"p": exp | q, "n": (1 << (w - 1)) | exp | q, "pay": exp | q | 1 | (q >> 2) | (q >> 5),
         "s": exp | 1, "nspay": (1 << (w - 1)) | exp | 3}[kind]
    if v >= 1 << (w - 1):
        v -= 1 << w
    return torch.tensor([v], dtype=torch.int64).to(_IT[dt]).view(dt)[0]


def nan_inputs(dt):
    """(name, tensor, [(bits, gs, sym, per_channel) ...]) of the NaN-origin cases."""
    g = torch.Generator().manual_seed(777)
    rnd = lambda *s: torch.randn(*s, generator=g).to(dt)
    PS = [(b, 128, s, True) for b in (4, 8) for s in (False, True)]
    out = []
    # 17 rows x 3 groups of 128 (51 scales): one NaN origin per row
    x = rnd(17, 384)
    inf, ninf = float("inf"), float("-inf")
    x[0, 5] = nan_bits(dt, "p")
    x[1, 130] = nan_bits(dt, "n")
    x[2, 300] = nan_bits(dt, "pay")
    x[3, 0] = nan_bits(dt, "s")
    x[4, 127] = nan_bits(dt, "nspay")
    x[5, 10] = nan_bits(dt, "p"); x[5, 11] = inf                     # NaN next to +inf
    x[6, 200] = nan_bits(dt, "n"); x[6, 201] = ninf                  # -NaN next to -inf
    x[7, 0:128] = inf                                                # all +inf: inf - inf
    x[8, 128:256] = ninf                                             # all -inf
    x[9, 256] = inf; x[9, 300] = ninf                                # +-inf, no NaN
    x[10, 0:128] = nan_bits(dt, "p")                                 # all NaN
    x[11, 0] = nan_bits(dt, "p"); x[11, 127] = nan_bits(dt, "n")     # both signs
    x[12, 383] = nan_bits(dt, "pay")                                 # last element
    x[13, 0:128] = 0.0; x[13, 64] = nan_bits(dt, "p")                # NaN among zeros
    x[14, 128:256] = 2.5; x[14, 129] = nan_bits(dt, "s")             # NaN in a constant group
    out.append(("rows17x384", x, PS + [(4, gs, s, True) for gs in (32, 64, 100, 256) for s in (False, True)]))
    # scale tensors of 1, 7, 8, 9, 16, 17, 33 elements
    for R in (1, 7, 8, 9, 16, 17, 33):
        x = rnd(R, 128)
        x[0, 3] = nan_bits(dt, "p")
        x[R // 2, 64] = nan_bits(dt, "n")
        x[R - 1, 127] = nan_bits(dt, "pay")
        out.append((f"r{R}x128", x, PS))
    # NaN / inf in a zero-padded tail group (K = 300, gs 128: tail of 44 elements + 84 zeros)
    x = rnd(5, 300)
    x[0, 280] = nan_bits(dt, "p")
    x[1, 256:300] = inf                                             # all-inf tail: the padding is 0
    x[2, 299] = nan_bits(dt, "n")
    x[3, 260] = ninf
    out.append(("tail5x300", x, PS + [(4, 100, s, True) for s in (False, True)]))
    # group sizes 1, 2, 3 (one NaN per group: the element itself is the group's min and max)
    x = rnd(6, 12)
    x[0, 0] = nan_bits(dt, "p"); x[0, 5] = nan_bits(dt, "n"); x[0, 7] = nan_bits(dt, "pay")
    x[1, 1] = nan_bits(dt, "s"); x[1, 2] = nan_bits(dt, "nspay"); x[1, 11] = inf
    x[2, 3] = ninf; x[2, 4] = inf; x[2, 5] = ninf
    x[3, 6] = nan_bits(dt, "p"); x[3, 7] = inf
    out.append(("gsmall6x12", x, [(b, gs, s, True) for gs in (1, 2, 3) for b in (4, 8) for s in (False, True)]))
    # small-tensor path (numel < group_size): whole tensor / per row, n = 1 and n > 1
    SP = [(b, 128, s, pc) for b in (4, 8) for s in (False, True) for pc in (True, False)]
    for name, shape, marks in (
            ("sm_v1_p", (1,), [((0,), "p")]), ("sm_v1_n", (1,), [((0,), "n")]),
            ("sm_v1_pay", (1,), [((0,), "pay")]), ("sm_v1_s", (1,), [((0,), "s")]),
            ("sm_v1_inf", (1,), [((0,), "inf")]), ("sm_v1_ninf", (1,), [((0,), "ninf")]),
            ("sm_v5", (5,), [((2,), "pay")]), ("sm_v7_inf", (7,), [((i,), "inf") for i in range(7)]),
            ("sm_c6x1", (6, 1), [((0, 0), "p"), ((1, 0), "n"), ((2, 0), "pay"), ((3, 0), "inf"), ((4, 0), "nspay")]),
            ("sm_c3x4", (3, 4), [((0, 1), "p"), ((2, 3), "n")]),
            ("sm_c9x3", (9, 3), [((0, 0), "p"), ((4, 1), "pay"), ((8, 2), "n")] + [((5, i), "ninf") for i in range(3)]),
            ("sm_t2x3x4", (2, 3, 4), [((1, 2, 3), "pay")])):
        x = rnd(*shape)
        for idx, kind in marks:
            x[idx] = inf if kind == "inf" else (ninf if kind == "ninf" else nan_bits(dt, kind))
        out.append((name, x, SP))
    x = nan_bits(dt, "pay").clone()                                  # 0-d
    out.append(("sm_0d_pay", x, SP))
    return out


def main_nan():
    tensors, cases = {}, []
    for dn in ("bf16", "f16", "f32", "f64"):
        dt = DTYPES[dn]
        for sn, x, plist in nan_inputs(dt):
            in_key = f"in.{dn}.{sn}"
            xs = x.view(torch.int16) if dt == torch.bfloat16 else x
            tensors[in_key] = xs.contiguous().clone()
            for bits, gs, sym, pc in plist:
                name = f"{dn}.{sn}.{'sym' if sym else 'asym'}.b{bits}.g{gs}.pc{int(pc)}"
                params = dict(bits=bits, group_size=gs, symmetric=sym, per_channel=pc)
                rec, res = run_case(params, x)
                rec.update(name=name, params=params, shape=list(x.shape), dtype=str(x.dtype), input=in_key)
                if res is not None:
                    r, dq = res
                    for k in ("tensor_q", "scales", "zero_points"):
                        tensors[f"{name}.{k}"] = r[k].contiguous()
                    rec["out_shapes"] = {k: list(r[k].shape) for k in ("tensor_q", "scales", "zero_points")}
                    if dq is not None:
                        tensors[name + ".dq"] = dq.contiguous()
                cases.append(rec)
    save_file(tensors, os.path.join(HERE, "golden_nan.safetensors"))
    with open(os.path.join(HERE, "golden_nan.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py --nan", "torch": torch.__version__,
                   "reference": "shanefitch/AWQ-Converter src/awq_quantizer/quantization/awq.py",
                   "cases": cases}, f, indent=1, sort_keys=True)
    print("nan cases", len(cases), "bytes", os.path.getsize(os.path.join(HERE, "golden_nan.safetensors")))


if __name__ == "__main__":
    if "--nan" in sys.argv[1:]:
        main_nan()
    else:
        main()
