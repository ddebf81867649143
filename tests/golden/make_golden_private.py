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


if __name__ == "__main__":
    main()
