#!/usr/bin/env python3
"""The memory structure's own ceiling at a given footprint: awq_stream_ceiling (read N bytes in
4 KiB waves, write N / 4: the quantizer's read-dominant traffic with no arithmetic) and
awq_stream_copy, timed with HIP events over back-to-back launches, per input size.  Quotes
what ONE launch over a single tensor's bytes can reach (ramp and tail included), next to
the kernels' own times on that tensor.

  python scripts/ceiling_probe.py --mb 117.44,469.8,1024
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", default="117.440512,1073.741824")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    from awq_quantizer import _hip
    dev = torch.device("cuda", 0)
    _hip.require_device(dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    for mb in (float(v) for v in a.mb.split(",")):
        n = int(mb * 1e6) // 4096 * 4096
        src = torch.randn(n // 4, device=dev).view(torch.uint8)
        for name, dst_bytes, fn in (("read_write_quarter", n // 4, _hip.stream_ceiling),
                                    ("copy", n, _hip.stream_copy)):
            dst = torch.empty(dst_bytes, dtype=torch.uint8, device=dev)
            for _ in range(3):
                fn(src, dst, s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn(src, dst, s)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            moved = n + dst_bytes
            print(json.dumps({"probe": name, "read_bytes": n, "write_bytes": dst_bytes, "us": round(us, 2),
                              "TBs": round(moved / us / 1e6, 3), "frac_8TBs": round(moved / us / 1e6 / 8, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
