#!/usr/bin/env python3
"""Bit check of the clip search of one library build against the oracle (A/B builds of
awq_fast.hip): bf16 / fp16, 4 / 8 bit, sym / asym, the test_scale_search shapes.
  python scripts/ab_search_check.py <lib.so>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402

from awq_quantizer import _hip  # noqa: E402
from oracle import awq_oracle as orc  # noqa: E402

_hip.load_library(os.path.abspath(sys.argv[1]))
from awq_quantizer.quantization import AWQQuantizer  # noqa: E402
bad = 0
for dtype in (torch.bfloat16, torch.float16):
    for bits in (4, 8):
        for sym in (False, True):
            g = torch.Generator().manual_seed(17 + bits)
            x = (torch.randn(32, 1024, generator=g) * 0.05).to(dtype)
            x[0, 3] = 2.0
            q = AWQQuantizer(bits=bits, group_size=128, symmetric=sym, scale_method="search", device="cuda",
                             logger_level="ERROR")
            ref = orc.quantize(x, bits=bits, group_size=128, symmetric=sym, search=(20, 10))
            res = q.quantize(x)
            ok = torch.equal(res["tensor_q"], ref["tensor_q"]) and torch.equal(res["zero_points"], ref["zero_points"])
            nd = int((res["tensor_q"] != ref["tensor_q"]).sum())
            bad += not ok
            print(sys.argv[1].split("/")[-1], dtype, bits, sym, "OK" if ok else f"DIFF ({nd} elements)")
sys.exit(1 if bad else 0)
