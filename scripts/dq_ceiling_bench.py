#!/usr/bin/env python3
"""dequantize_packed (awq_dequant_batch_kernel) against its measured ceiling, interleaved in one
process: the product kernel, diagnostics-build variants (tuning dq_words_v1) and
awq_dequant_ceiling (the same 1 : 8 read : write structure without arithmetic or parameter
loads) on the same footprint, `--rounds` rounds of `--iters` launches each; medians per case.
Default: the Llama-3-8B lm_head, 128256 x 4096, gs 128, 4-bit (2.1 GB of fp32 output, past the
256 MiB Infinity Cache).

  python scripts/dq_ceiling_bench.py --variants 0,10,11
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402

from awq_quantizer import _hip  # noqa: E402
from awq_quantizer.quantization import AWQQuantizer  # noqa: E402


def timed(fn, iters):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=128256)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--group-size", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default="", help="diagnostics-build dq_words_v1 values (0 = its default)")
    a = ap.parse_args()
    torch.manual_seed(0)
    x = (torch.randn(a.rows, a.K, device="cuda") * 0.02).bfloat16()
    q = AWQQuantizer(bits=4, group_size=a.group_size, symmetric=False, logger_level="ERROR")
    p = q.quantize_packed(x)
    del x
    n = a.rows * a.K
    G = a.K // a.group_size
    alg = n * 4 + n // 2 + a.rows * G * 2 + a.rows * -(-G // 8) * 4
    out = torch.empty((a.rows, a.K), dtype=torch.float32, device="cuda")
    ref = q.dequantize_packed(p).clone()
    stream = torch.cuda.current_stream().cuda_stream
    rows, K, L = a.rows, a.K, a.group_size

    def product():
        _hip.dequantize_packed(p["qweight"], p["qzeros"], p["scales"], rows, K, L, 4, False, out)

    cases = {"product": product,
             "ceiling": lambda: _hip.dequant_ceiling(p["qweight"], out, stream)}
    for v in [int(t) for t in a.variants.split(",") if t != ""]:
        def variant(v=v):
            with _hip.tuning(dq_words_v1=v):
                _hip.dequantize_packed(p["qweight"], p["qzeros"], p["scales"], rows, K, L, 4, False, out)
        cases[f"diag_v{v}"] = variant
    same = {}
    for name, fn in cases.items():     # warm-up + bits check of every dequantize case
        fn()
        torch.cuda.synchronize()
        if name != "ceiling":
            same[name] = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
    times = {k: [] for k in cases}
    for r in range(a.rounds):
        for name, fn in cases.items():
            times[name].append(timed(fn, a.iters))
    ceil_us = statistics.median(times["ceiling"])
    for name, ts in times.items():
        us = statistics.median(ts)
        print(json.dumps({"case": name, "rows": rows, "K": K, "group_size": L, "us_median": round(us, 1),
                          "us_min": round(min(ts), 1), "us_max": round(max(ts), 1),
                          "TBs_algorithmic": round(alg / us / 1e6, 3), "frac_8TBs": round(alg / us / 8e6, 4),
                          "of_ceiling": round(ceil_us / us, 4), "same_bits": same.get(name)}), flush=True)


if __name__ == "__main__":
    main()
