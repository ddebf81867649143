#!/usr/bin/env python3
"""Throughput of the single-tensor entry point (awq_quantize_groups / awq_quantize_search)
per input dtype: bf16 takes the streaming kernel, fp16/fp32 the generic one.

  python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16,f16,f32
  python scripts/generic_bench.py --shape "1024,4096;4096,4096" --dtypes bf16   (";" separates shapes)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402

DT = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="14336,4096")
    ap.add_argument("--dtypes", default="bf16,f16,f32")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--search", type=int, default=0, help="clip-search candidates (0 = RTN)")
    args = ap.parse_args()
    from awq_quantizer import _hip
    dev = torch.device("cuda", 0)
    _hip.require_device(dev)
    for shape in args.shape.split(";"):
        for name in args.dtypes.split(","):
            one(args, _hip, dev, shape, name)


def one(args, _hip, dev, shape, name):
    R, K = (int(v) for v in shape.split(","))
    G = K // 128
    x = (torch.randn(R, K, device=dev) * 0.02).to(DT[name])
    qw = torch.empty(R, K // 8, dtype=torch.int32, device=dev)
    qz = torch.empty(R, -(-G // 8), dtype=torch.int32, device=dev)
    sc = torch.empty(R, G, dtype=torch.float16, device=dev)
    stage = {}
    if args.search or not _hip.ragged_eligible(DT[name], R, K, 128):
        stage = dict(tensor_q=torch.empty(R * K, dtype=torch.int32, device=dev),
                     zeros=torch.empty(R, G, dtype=torch.int32, device=dev))

    def run():
        if args.search:
            _hip.quantize_search(x, R, K, 128, 4, False, 20, args.search, qweight=qw, qzeros=qz, scales=sc,
                                 **stage)
        else:
            _hip.quantize_groups(x, R, K, 128, 4, False, qweight=qw, qzeros=qz, scales=sc, **stage)
    for _ in range(3):
        run()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(args.iters):
        run()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / args.iters * 1e3
    nbytes = x.numel() * x.element_size()
    print(json.dumps({"dtype": name, "shape": [R, K], "search": args.search, "us": round(us, 1),
                      "input_GBs": round(nbytes / us / 1e3, 1)}))


if __name__ == "__main__":
    main()
