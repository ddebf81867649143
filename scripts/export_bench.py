#!/usr/bin/env python3
"""Throughput of the AutoAWQ "GEMM"-layout export (include/awq_hip.h awq_export_autoawq_gemm,
csrc/awq_export.hip) on Llama-3-8B linear shapes: a packed 4-bit weight
[N, K] (qweight N x K/8, qzeros N x G/8, scales N x G) rewritten as qweight [K, N/8], qzeros
[G, N/8], scales [G, N].  Bytes moved = every input word read once + every output word
written once; quoted against 8 TB/s and against awq_stream_copy of the same byte count
(the memory system's copy rate for this size).

  python scripts/export_bench.py [--iters 20] [--lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_X.so]
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402

SHAPES = {"q_proj/o_proj": (4096, 4096), "k_proj/v_proj": (1024, 4096), "gate/up_proj": (14336, 4096),
          "down_proj": (4096, 14336), "lm_head": (128256, 4096)}


def timed(fn, iters):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default=None, help="A/B build of the library (scripts/build_variant.sh)")
    args = ap.parse_args()
    from awq_quantizer import _hip
    if args.lib:
        _hip.load_library(os.path.join(ROOT, args.lib))
    from awq_quantizer.quantization import AWQQuantizer
    dev = torch.device("cuda", 0)
    _hip.require_device(dev)
    q = AWQQuantizer(bits=4, group_size=128, symmetric=False, device="cuda", logger_level="ERROR")
    for name, (N, K) in SHAPES.items():
        g = torch.Generator(device=dev).manual_seed(N + K)
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).bfloat16()
        pk = q.quantize_packed(w)
        del w
        t_us = timed(lambda: q.export_autoawq(pk), args.iters)
        out = q.export_autoawq(pk)
        nbytes = sum(pk[k].numel() * pk[k].element_size() for k in ("qweight", "qzeros", "scales")) + \
            sum(out[k].numel() * out[k].element_size() for k in ("qweight", "qzeros", "scales"))
        half = (nbytes // 2 + 15) // 16 * 16      # copy of the same read + write volume
        src = torch.empty(half, dtype=torch.uint8, device=dev)
        dst = torch.empty_like(src)
        t_copy = timed(lambda: _hip.stream_copy(src, dst, _hip.stream_ptr(dev)), args.iters)
        sha = hashlib.sha256(b"".join(out[k].cpu().contiguous().view(torch.uint8).numpy().tobytes() for k in ("qweight", "qzeros", "scales")))
        print(json.dumps({"lib": args.lib or "product", "tensor": name, "N": N, "K": K, "us": round(t_us, 1), "bytes": nbytes,
                          "GBs": round(nbytes / t_us / 1e3, 1), "frac_8TBs": round(nbytes / t_us / 1e3 / 8000, 3),
                          "copy_us": round(t_copy, 1),
                          "frac_of_copy": round(t_copy / t_us, 3), "out_sha": sha.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
