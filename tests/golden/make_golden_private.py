#!/usr/bin/env python3
"""Golden fixtures for the reference quantizer's PRIVATE methods, which subclasses and
callers of the reference reach into (TEST INFRASTRUCTURE ONLY, like make_golden.py):

  _compute_scale_zp_for_group  awq.py:173-213     _calculate_scale_zp  awq.py:130-171
  _quantize_tensor             awq.py:215-250     _dequantize_tensor   awq.py:252-284
  _quantize_per_group          awq.py:286-374

Imports the reference from /root/reference in THIS container, runs each method on CPU and
writes inputs + outputs as data:

  tests/golden/golden_private.safetensors   every input and output tensor, native dtypes
  tests/golden/golden_private.json          per-call method, parameters and tensor keys

Re-run with:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_private.py

--promote (round 5): calls of _quantize_tensor / _dequantize_tensor whose parameters promote
the tensor's dtype or broadcast it other than per channel -> golden_promote.{safetensors,json}
(main_promote below).
"""
import json
import logging
import os
import sys

REF_SRC = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))
if not os.path.isdir(REF_SRC):
    sys.exit("make_golden_private.py: /root/reference is absent (fixtures are generated in the build container)")
sys.dont_write_bytecode = True
sys.path.insert(0, REF_SRC)

import torch  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

from awq_quantizer.quantization.awq import AWQQuantizer  # noqa: E402  (reference)

sys.path.insert(0, HERE)
from make_golden import edge_rows_f32, rand_input  # noqa: E402

logging.disable(logging.CRITICAL)
torch.set_num_threads(8)
DTYPES = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32, "f64": torch.float64}


def main():
    tensors, calls = {}, []

    def put(key, t):
        tensors[key] = t.detach().contiguous().clone()
        return key

    n = 0
    for dn, dt in DTYPES.items():
        edge = edge_rows_f32().to(dt)
        inputs = {"edge16x256": edge, "r8x300": rand_input((8, 300), 21, dt), "v1000": rand_input((1000,), 22, dt, 0.02),
                  "t3x4x50": rand_input((3, 4, 50), 23, dt), "s10x10": rand_input((10, 10), 24, dt),
                  "v60": rand_input((60,), 25, dt)}
        for bits in (4, 8):
            for sym in (False, True):
                for pc in (True, False):
                    params = {"bits": bits, "group_size": 32 if dn == "f32" else 128, "symmetric": sym,
                              "per_channel": pc}
                    q = AWQQuantizer(device="cpu", **params)
                    for name, x in inputs.items():
                        base = f"{dn}.b{bits}.{'sym' if sym else 'asym'}.{'pc' if pc else 'pt'}.{name}"
                        xk = put(f"in.{dn}.{name}", x)
                        # _quantize_per_group (large path, or the small path when numel < group_size)
                        tq, s, z = q._quantize_per_group(x)
                        calls.append({"method": "_quantize_per_group", "params": params, "dtype": dn, "x": xk,
                                      "out": [put(f"{base}.qpg.tq", tq), put(f"{base}.qpg.s", s),
                                              put(f"{base}.qpg.z", z)]})
                        # _calculate_scale_zp + _quantize_tensor + _dequantize_tensor on the whole tensor
                        s2, z2 = q._calculate_scale_zp(x)
                        q2 = q._quantize_tensor(x, s2, z2)
                        d2 = q._dequantize_tensor(q2, s2, z2)
                        calls.append({"method": "_calculate_scale_zp", "params": params, "dtype": dn, "x": xk,
                                      "out": [put(f"{base}.csz.s", s2), put(f"{base}.csz.z", z2)]})
                        calls.append({"method": "_quantize_tensor", "params": params, "dtype": dn, "x": xk,
                                      "scale": f"{base}.csz.s", "zero_point": f"{base}.csz.z",
                                      "out": [put(f"{base}.qt", q2)]})
                        calls.append({"method": "_dequantize_tensor", "params": params, "dtype": dn,
                                      "x": f"{base}.qt", "scale": f"{base}.csz.s", "zero_point": f"{base}.csz.z",
                                      "out": [put(f"{base}.dqt", d2)]})
                        n += 4
                    # _compute_scale_zp_for_group on single groups: every edge row (NaN, inf,
                    # constant, signed zeros, ...) and a random group
                    if pc:
                        for i in range(edge.shape[0]):
                            g = edge[i, :128]
                            s3, z3 = q._compute_scale_zp_for_group(g)
                            k = f"{dn}.b{bits}.{'sym' if sym else 'asym'}.edge{i}"
                            calls.append({"method": "_compute_scale_zp_for_group", "params": params, "dtype": dn,
                                          "x": put(f"in.{dn}.edge{i}", g),
                                          "out": [put(f"{k}.csg.s", s3), put(f"{k}.csg.z", z3)]})
                            n += 1
    save_file(tensors, os.path.join(HERE, "golden_private.safetensors"))
    with open(os.path.join(HERE, "golden_private.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_private.py", "torch": torch.__version__,
                   "reference": "shanefitch/AWQ-Converter src/awq_quantizer/quantization/awq.py:130-374",
                   "calls": calls}, f, indent=0)
    print(f"{n} calls, {len(tensors)} tensors")


def promote_variants(x, s, z, gen):
    """(name, scale, zero_point) parameter sets for the dtype-promotion / broadcast fixtures:
    the reference's own parameters cast to every dtype, jittered off the narrow dtypes'
    grids (so 'enters at its own value' and 'rounded to the op dtype' give different bits),
    one-element and 0-d forms, integer zero points, mixed scale / zero dtypes, and broadcasts
    that are not per-channel."""
    jit = lambda t: t.double() * (1 + (torch.rand(t.shape, generator=gen, dtype=torch.float64) - 0.5) * 2 ** -7)
    first = lambda t: t.reshape(-1)[:1]
    out = []
    for pn, pdt in DTYPES.items():
        if pdt != x.dtype:
            out.append((f"cast_{pn}", s.to(pdt), z.to(pdt)))
        out.append((f"jit_{pn}", jit(s).to(pdt), z.to(pdt)))
        out.append((f"0d_{pn}", jit(first(s)).reshape(()).to(pdt), first(z).reshape(()).to(pdt)))
        out.append((f"1el_{pn}", jit(first(s)).to(pdt), first(z).to(pdt)))
    out.append(("z_i32", jit(s).float(), z.to(torch.int32)))
    out.append(("z_i64_0d", jit(first(s)).reshape(()).half(), torch.tensor(3, dtype=torch.int64)))
    out.append(("s_f16_z_bf16", jit(s).half(), z.bfloat16()))
    out.append(("s_bf16_z_f64", jit(s).bfloat16(), z.double()))
    if x.dim() >= 2:
        R, C = x.shape[0], x.shape[-1]
        col = lambda n, dt: (0.01 + torch.rand(n, generator=gen, dtype=torch.float64) * 0.05).to(dt)
        zc = lambda n, dt: torch.randint(0, 15, (n,), generator=gen).to(dt)
        out.append(("bc_rowcol_f32", col(R, torch.float32).reshape([R] + [1] * (x.dim() - 1)),
                    zc(R, torch.float32).reshape([R] + [1] * (x.dim() - 1))))
        out.append(("bc_lastdim_own", col(C, x.dtype), zc(C, x.dtype)))
        out.append(("bc_lastdim_f64", col(C, torch.float64), zc(C, torch.int32)))
        out.append(("bc_1xC_Rx1", col(C, x.dtype).reshape(1, C) if x.dim() == 2 else col(C, x.dtype),
                    zc(R, torch.float16).reshape([R] + [1] * (x.dim() - 1))))
        out.append(("bc_elem_i32z", jit(first(s)).reshape(()).float(),
                    torch.randint(0, 15, tuple(x.shape), generator=gen, dtype=torch.int32)))
        out.append(("bad_rows", col(R + 1, torch.float32), zc(R + 1, torch.float32)))
    else:
        out.append(("bc_grow_4x1", (0.01 + torch.rand(4, 1, generator=gen) * 0.05).to(x.dtype),
                    torch.randint(0, 15, (4, 1), generator=gen).to(torch.float32)))
    return out


def main_promote():
    """Reference calls of _quantize_tensor / _dequantize_tensor whose parameters promote the
    tensor's dtype (awq.py:245 tensor / scale + zero_point, awq.py:282 (tensor_q - zero_point)
    * scale evaluated with torch's type promotion) or broadcast it other than per channel,
    plus int32 tensor_q (quantize()'s dtype) dequantized with float parameters.  Calls that
    raise in the reference are recorded with the exception type.
      tests/golden/golden_promote.safetensors / golden_promote.json"""
    tensors, calls = {}, []
    gen = torch.Generator().manual_seed(5150)

    def put(key, t):
        tensors[key] = t.detach().contiguous().clone()
        return key

    def rec(method, params, xk, sk, zk, fn, out_key):
        c = {"method": method, "params": params, "x": xk, "scale": sk, "zero_point": zk}
        try:
            c["out"] = [put(out_key, fn())]
        except Exception as e:   # the reference raises: record the behaviour
            c["raises"] = type(e).__name__
            c["message"] = str(e)
        calls.append(c)
        return c

    qparams = [{"bits": 4, "group_size": 128, "symmetric": False, "per_channel": True},
               {"bits": 4, "group_size": 128, "symmetric": False, "per_channel": False},
               {"bits": 8, "group_size": 128, "symmetric": True, "per_channel": True}]
    for dn, dt in DTYPES.items():
        edge = edge_rows_f32()[:8, 100:124].to(dt)
        inputs = {"edge8x24": edge, "r6x24": rand_input((6, 24), 31, dt), "t3x2x8": rand_input((3, 2, 8), 32, dt),
                  "v40": rand_input((40,), 33, dt, 0.02)}
        for qi, params in enumerate(qparams):
            q = AWQQuantizer(device="cpu", **params)
            for name, x in inputs.items():
                if name == "edge8x24" and qi != 0:
                    continue
                xk = put(f"in.{dn}.{name}", x)
                s, z = q._calculate_scale_zp(x)
                for vn, sv, zv in promote_variants(x, s, z, gen):
                    base = f"{dn}.q{qi}.{name}.{vn}"
                    sk, zk = put(f"{base}.s", sv), put(f"{base}.z", zv)
                    c = rec("_quantize_tensor", params, xk, sk, zk, lambda: q._quantize_tensor(x, sv, zv), f"{base}.qt")
                    if "out" not in c:
                        continue
                    q2 = tensors[c["out"][0]]
                    rec("_dequantize_tensor", params, c["out"][0], sk, zk, lambda: q._dequantize_tensor(q2, sv, zv),
                        f"{base}.dqt")
                    qi32 = put(f"{base}.qt_i32", torch.nan_to_num(q2.double(), nan=0.0).to(torch.int32))
                    rec("_dequantize_tensor", params, qi32, sk, zk,
                        lambda: q._dequantize_tensor(tensors[qi32], sv, zv), f"{base}.dqt_i32")
    save_file(tensors, os.path.join(HERE, "golden_promote.safetensors"))
    with open(os.path.join(HERE, "golden_promote.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_private.py --promote", "torch": torch.__version__,
                   "reference": "shanefitch/AWQ-Converter src/awq_quantizer/quantization/awq.py:215-284",
                   "calls": calls}, f, indent=0)
    raised = sum("raises" in c for c in calls)
    print(f"{len(calls)} calls ({raised} raise), {len(tensors)} tensors")


INT_DTYPES = {"i64": torch.int64, "i32": torch.int32, "i16": torch.int16, "i8": torch.int8, "u8": torch.uint8,
              "bool": torch.bool, "u16": torch.uint16, "u32": torch.uint32, "u64": torch.uint64}
# int64 values whose conversions round twice (int64 -> fp32 -> bf16 at a bf16 tie, fp32 ties,
# beyond 2^53) and the int64 extremes
I64_SPECIAL = [2 ** 30 + 2 ** 22 + 1, -(2 ** 30 + 2 ** 22 + 1), 2 ** 62 + 2 ** 38 + 1, 2 ** 53 + 1, 2 ** 24 + 1,
               -(2 ** 24 + 3), -2 ** 63, 2 ** 63 - 1, 2 ** 40 + 2 ** 32 + 1, 65519, 65520, -65536]


def int_inputs(dt, gen):
    """Integer / bool tensors: tensor_q-like values, the dtype's full range (int64: with the
    double-rounding and extreme values above), 3-D, 1-D, 0-d and one-element forms."""
    if dt == torch.bool:
        rnd = lambda shape: torch.randint(0, 2, shape, generator=gen).bool()
        full = rnd
    else:
        info = torch.iinfo(dt)
        lo, hi = max(info.min, -2 ** 62), min(info.max, 2 ** 62)

        def full(shape):
            if dt == torch.uint64:     # the whole 64-bit range, values >= 2^63 included
                v = torch.randint(-2 ** 62, 2 ** 62, shape, generator=gen, dtype=torch.int64) * 2
                return v.view(torch.uint64)
            return torch.randint(lo, hi, shape, generator=gen, dtype=torch.int64).to(dt)

        def rnd(shape):
            return torch.randint(0 if info.min == 0 else -8, 16, shape, generator=gen).to(dt)
    w = full((6, 24))
    if dt == torch.int64:
        w.view(-1)[:len(I64_SPECIAL)] = torch.tensor(I64_SPECIAL, dtype=torch.int64)
    out = {"q6x24": torch.randint(0, 2 if dt == torch.bool else 16, (6, 24), generator=gen).to(dt), "w6x24": w,
           "v40": full((40,)), "s0d": rnd(()), "e1": full((1,))}
    if dt in (torch.int64, torch.int8):
        out["t3x2x8"] = rnd((3, 2, 8))
    return out


def int_variants(x, s, z, gen):
    """(name, scale, zero_point) for integer tensors: float parameters per channel / 0-d /
    one-element in every float dtype (jittered off the narrow grids), integer and bool
    parameters (int / int true division, integer ops that wrap, exact int64 beyond 2^53),
    and non-per-channel broadcasts."""
    jit = lambda t: t.double() * (1 + (torch.rand(t.shape, generator=gen, dtype=torch.float64) - 0.5) * 2 ** -7)
    first = lambda t: t.reshape(-1)[:1]
    out = []
    for pn, pdt in DTYPES.items():
        out.append((f"pc_{pn}", jit(s).to(pdt), z.to(pdt)))
        out.append((f"0d_{pn}", jit(first(s)).reshape(()).to(pdt), first(z).reshape(()).to(pdt)))
        out.append((f"1el_{pn}", jit(first(s)).to(pdt), first(z).to(pdt)))
    R = s.numel()
    out.append(("z_i64", jit(s).float(), z.to(torch.int64)))
    out.append(("z_i8_0d", jit(first(s)).reshape(()).bfloat16(), torch.tensor(3, dtype=torch.int8)))
    out.append(("z_u8", jit(s).half(), z.to(torch.uint8)))
    out.append(("z_i16_1el", jit(first(s)).bfloat16(), torch.tensor([-300], dtype=torch.int16)))
    out.append(("si64_zi64_0d", torch.tensor(2, dtype=torch.int64), torch.tensor(5, dtype=torch.int64)))
    out.append(("si16_zi16", torch.randint(1, 6, s.shape, generator=gen).to(torch.int16),
                torch.randint(-3, 4, s.shape, generator=gen).to(torch.int16)))
    out.append(("si8_zu8", torch.randint(-5, 6, s.shape, generator=gen).to(torch.int8),
                torch.randint(0, 200, s.shape, generator=gen).to(torch.uint8)))
    out.append(("big_i64_0d", torch.tensor(3, dtype=torch.int64), torch.tensor(2 ** 62 + 2 ** 38 + 1, dtype=torch.int64)))
    out.append(("big_i64_pc", torch.tensor([-(2 ** 61) - 7] * R, dtype=torch.int64).reshape(s.shape),
                torch.tensor([2 ** 55 + 3] * R, dtype=torch.int64).reshape(s.shape)))
    out.append(("z_bool_0d", jit(first(s)).reshape(()).float(), torch.tensor(True)))
    out.append(("s_bool_z_f16", torch.ones(s.shape, dtype=torch.bool), z.half()))
    if x.dim() >= 2:
        C = x.shape[-1]
        col = lambda n, dt: (0.01 + torch.rand(n, generator=gen, dtype=torch.float64) * 0.05).to(dt)
        out.append(("bc_lastdim_f32_i32", col(C, torch.float32), torch.randint(0, 15, (C,), generator=gen).int()))
        out.append(("bc_lastdim_i64", torch.randint(1, 9, (C,), generator=gen), torch.randint(-9, 9, (C,),
                                                                                               generator=gen)))
    return out


def main_promote_int():
    """Reference calls of _quantize_tensor / _dequantize_tensor on INTEGER and bool tensors
    (awq.py:245 / :282 evaluated for any tensor dtype: int64 / int32 / int16 / int8 / uint8 /
    bool / uint16 / uint32 / uint64) with float, integer and bool parameters in per-channel,
    0-d, one-element and broadcast forms.  Calls that raise in the reference are recorded with
    the exception type.
      tests/golden/golden_promote_int.safetensors / golden_promote_int.json"""
    tensors, calls = {}, []
    gen = torch.Generator().manual_seed(6160)

    def put(key, t):
        tensors[key] = t.detach().contiguous().clone()
        return key

    def rec(method, params, xk, sk, zk, fn, out_key):
        c = {"method": method, "params": params, "x": xk, "scale": sk, "zero_point": zk}
        try:
            c["out"] = [put(out_key, fn())]
        except Exception as e:   # the reference raises: record the behaviour
            c["raises"] = type(e).__name__
            c["message"] = str(e)
        calls.append(c)

    qparams = [{"bits": 4, "group_size": 128, "symmetric": False, "per_channel": True},
               {"bits": 8, "group_size": 128, "symmetric": True, "per_channel": False}]
    for dn, dt in INT_DTYPES.items():
        for name, x in int_inputs(dt, gen).items():
            xk = put(f"in.{dn}.{name}", x)
            # realistic parameters: the reference's own per-channel scale / zero point of a
            # float tensor of x's shape (values near tensor_q's range)
            xf = torch.randn(tuple(x.shape), generator=torch.Generator().manual_seed(41))
            for qi, params in enumerate(qparams):
                q = AWQQuantizer(device="cpu", **params)
                s, z = q._calculate_scale_zp(xf)
                for vn, sv, zv in int_variants(x, s, z, gen):
                    base = f"{dn}.q{qi}.{name}.{vn}"
                    sk, zk = put(f"{base}.s", sv), put(f"{base}.z", zv)
                    rec("_quantize_tensor", params, xk, sk, zk, lambda: q._quantize_tensor(x, sv, zv), f"{base}.qt")
                    rec("_dequantize_tensor", params, xk, sk, zk, lambda: q._dequantize_tensor(x, sv, zv),
                        f"{base}.dqt")
    save_file(tensors, os.path.join(HERE, "golden_promote_int.safetensors"))
    with open(os.path.join(HERE, "golden_promote_int.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_private.py --promote-int", "torch": torch.__version__,
                   "reference": "shanefitch/AWQ-Converter src/awq_quantizer/quantization/awq.py:215-284",
                   "calls": calls}, f, indent=0)
    raised = sum("raises" in c for c in calls)
    print(f"{len(calls)} calls ({raised} raise), {len(tensors)} tensors")


if __name__ == "__main__":
    if "--promote-int" in sys.argv[1:]:
        main_promote_int()
    elif "--promote" in sys.argv[1:]:
        main_promote()
    else:
        main()
