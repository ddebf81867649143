#!/usr/bin/env python3
"""Workload for the dequantize_packed counter passes (rocprofv3 --pmc): quantize one
[rows, K] bf16 tensor (default the Llama-3-8B lm_head, 128256 x 4096, gs 128) with
quantize_packed, then time dequantize_packed `--iters` times with HIP events; prints one
JSON line.  Used by scripts/cmd/r6e.sh; the kernel of interest is awq_dequant_batch_kernel."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402

from awq_quantizer.quantization import AWQQuantizer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=128256)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--group-size", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    torch.manual_seed(0)
    x = (torch.randn(a.rows, a.K, device="cuda") * 0.02).bfloat16()
    q = AWQQuantizer(bits=4, group_size=a.group_size, symmetric=False, logger_level="ERROR")
    p = q.quantize_packed(x)
    del x
    q.dequantize_packed(p)   # warm-up
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(a.iters):
        q.dequantize_packed(p)
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3 / a.iters
    n = a.rows * a.K
    alg = n * 4 + n // 2 + a.rows * (a.K // a.group_size) * 2 + a.rows * -(-(a.K // a.group_size) // 8) * 4
    print(json.dumps({"rows": a.rows, "K": a.K, "group_size": a.group_size, "us": round(us, 1),
                      "algorithmic_bytes": alg, "TBs": round(alg / us / 1e6, 3), "frac_8TBs": round(alg / us / 8e6, 4)}))


if __name__ == "__main__":
    main()
