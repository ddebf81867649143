#!/usr/bin/env python3
"""One large tensor per launch (quantize_packed per tensor, the CLI's per-batch launches):
per-launch time of awq_quantize_groups on one [rows, K] tensor, each launch bracketed by its
own HIP events, in three clock states —
  idle:   after 0.5 s with the GPU idle;
  warm:   right after ~200 ms of streaming (awq_stream_ceiling), the clocks settled;
  paired: the tensor launched between launches of the whole Llama-3-8B set (one ragged launch),
          so the chip streams continuously.
Prints one JSON line per (shape, state): median / min per launch, the first launch's time,
and the fraction of 8 TB/s for the algorithmic bytes (2.51953 B per bf16 element at gs 128).

  python scripts/single_launch_bench.py --shapes "128256,4096;4096,14336"
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402

import bench  # noqa: E402  (tensor-set manifests)


def per_launch(fn, n):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) * 1e3 for a, b in evs]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="128256,4096;4096,14336")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default="")
    a = ap.parse_args()
    from awq_quantizer import _hip
    from awq_quantizer.quantization.batch import PackedBatch
    if a.lib:
        _hip.load_library(a.lib)
    dev = torch.device("cuda", 0)
    _hip.require_device(dev)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    stream = torch.cuda.current_stream().cuda_stream
    # ~200 ms of streaming for the warm state
    buf = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    sink = torch.empty(1 << 28, dtype=torch.uint8, device=dev)

    def settle(ms=200.0):
        t0 = time.time()
        while (time.time() - t0) * 1e3 < ms:
            for _ in range(8):
                _hip.stream_ceiling(buf, sink, stream)
            torch.cuda.synchronize()

    g = torch.Generator(device=dev)
    set_inputs = {}
    for i, s in enumerate(bench.shapes_of("llama3-8b")):
        g.manual_seed(i)
        set_inputs[f"t{i}"] = (torch.randn(*s, generator=g, device=dev) * 0.02).to(dt)
    whole = PackedBatch(set_inputs, bits=4, symmetric=False)
    whole.run()
    set_elems = sum(t.numel() for t in set_inputs.values())
    for shp in a.shapes.split(";"):
        R, K = (int(v) for v in shp.split(","))
        g.manual_seed(99)
        x = (torch.randn(R, K, generator=g, device=dev) * 0.02).to(dt)
        qw = torch.empty((R, K // 8), dtype=torch.int32, device=dev)
        qz = torch.empty((R, K // 128 // 8 + (1 if (K // 128) % 8 else 0)), dtype=torch.int32, device=dev)
        sc = torch.empty((R, K // 128), dtype=torch.float16, device=dev)
        one = lambda: _hip.quantize_groups(x, R, K, 128, 4, False, qweight=qw, qzeros=qz, scales=sc)
        one()
        torch.cuda.synchronize()
        alg = R * K * (2 + 0.5 + 2 / 128 + 0.5 / 128)
        res = {}
        time.sleep(0.5)
        res["idle"] = per_launch(one, a.iters)
        settle()
        res["warm"] = per_launch(one, a.iters)
        paired, whole_t = [], []
        for _ in range(a.iters):
            w = per_launch(whole.run, 1)
            whole_t += w
            paired += per_launch(one, 1)
        res["paired"] = paired
        for state, ts in res.items():
            med = statistics.median(ts)
            print(json.dumps({"shape": [R, K], "dtype": a.dtype, "state": state, "us_median": round(med, 2),
                              "us_min": round(min(ts), 2), "us_first": round(ts[0], 2),
                              "frac_8TBs_median": round(alg / med / 8e6, 4), "frac_8TBs_best": round(alg / min(ts) / 8e6, 4)}),
                  flush=True)
        wm = statistics.median(whole_t)
        print(json.dumps({"set": "llama3-8b", "state": "paired", "us_median": round(wm, 1),
                          "frac_8TBs_median": round(set_elems * 2.51953 / wm / 8e6, 4)}), flush=True)


if __name__ == "__main__":
    main()
