#!/usr/bin/env python3
"""Sustained-load probe: per-launch durations (HIP events on the stream) of the bench's
quantize kernel and of the library's stream-copy kernel over long back-to-back runs, to
separate power/clock management effects from kernel behaviour.

  python scripts/sustain_probe.py --launches 2000
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def timed(fn, n, stream):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for i in range(n):
        ev[i][0].record(stream)
        fn(i)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) * 1e3 for a, b in ev]


def summary(us, width=100):
    out = []
    for i in range(0, len(us), width):
        blk = sorted(us[i:i + width])
        out.append(round(blk[len(blk) // 2], 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=2000)
    ap.add_argument("--workload", default="opt-125m")
    args = ap.parse_args()
    from awq_quantizer import _hip
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device("cuda", 0)
    _hip.require_device(dev)
    stream = torch.cuda.current_stream(dev)
    shapes = bench.shapes_of(args.workload)
    batches = [PackedBatch(bench.make_set(shapes, r * 100003, dev), bits=4, symmetric=False) for r in range(5)]
    src = torch.empty(315670480 // 4, dtype=torch.int32, device=dev).fill_(1)   # same bytes as one launch
    dst = torch.empty_like(src)
    torch.cuda.synchronize()
    q = timed(lambda i: batches[i % 5].run(stream), args.launches, stream)
    print(json.dumps({"kernel": "awq_fast_kernel", "median_us_per_100_launches": summary(q)}), flush=True)
    c = timed(lambda i: _hip.stream_copy(src, dst, stream.cuda_stream), args.launches, stream)
    print(json.dumps({"kernel": "awq_stream_copy (315.7 MB read+write)", "median_us_per_100_launches": summary(c)}),
          flush=True)
    q2 = timed(lambda i: batches[i % 5].run(stream), args.launches, stream)
    print(json.dumps({"kernel": "awq_fast_kernel (again, after the copy run)", "median_us_per_100_launches": summary(q2)}),
          flush=True)


if __name__ == "__main__":
    main()
