#!/usr/bin/env python3
"""Per-wave timeline of one ragged launch (build variant AWQ_TRACE: every wave records
s_memrealtime at start, when its tile's loads are issued, when they have landed, and at
the end).

  make -C awq-converter_amd/csrc variant-trace VFLAGS=-DAWQ_TRACE
  python scripts/trace_waves.py --set opt-125m

Prints the launch span, the median wave lifetime split into setup (start -> loads
issued: kernel arguments, tensor table / descriptor loads, tile geometry), load wait
(issued -> landed) and compute + store issue (landed -> end), and the mean number of
live waves (sum of lifetimes / span; 8192 = every slot of the chip busy).
The kernel must run its default one-wave-per-tile grid (no AWQ_HIP_* overrides): the
trace buffer holds exactly one record per wave of that grid.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402

import kbench  # noqa: E402  (tensor-set manifests)

TICK_US = 0.01   # s_memrealtime: 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="opt-125m")
    ap.add_argument("--lib", default=os.path.join(ROOT, "awq-converter_amd/awq_quantizer/_lib/variants/libawq_hip_trace.so"))
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from awq_quantizer import _hip
    from awq_quantizer.quantization.batch import PackedBatch
    _hip.load_library(args.lib)          # the AWQ_TRACE build, explicitly (first load decides)
    raw = ctypes.CDLL(args.lib)
    dev = torch.device("cuda", 0)
    _hip.require_device(dev)
    shapes = kbench.shapes_of(args.set)
    g = torch.Generator(device=dev)
    batches = []
    for r in range(args.reps):
        inputs = {}
        for i, s in enumerate(shapes):
            g.manual_seed(r * 1000 + i)
            inputs[f"t{i}"] = (torch.randn(*s, generator=g, device=dev) * 0.02).to(torch.bfloat16)
        batches.append(PackedBatch(inputs, bits=4, symmetric=False))
    # one wave per tile: the kernel writes 4 words for every wave of the grid
    nwaves = -(-max(b.total_tiles for b in batches) // 4) * 4
    buf = torch.zeros(nwaves * 4, dtype=torch.int64, device=dev)
    assert raw.awq_debug_set_trace(ctypes.c_void_p(buf.data_ptr())) == 0
    for it in range(3 * args.reps):
        buf.zero_()
        b = batches[it % args.reps]
        b.run()
        torch.cuda.synchronize()
        if it < args.reps:
            continue
        tr = buf.view(nwaves, 4)[: b.total_tiles].cpu().double()
        t0 = tr[:, 0].min()
        start, issued, landed, end = [(tr[:, i] - t0) * TICK_US for i in range(4)]
        span = float(end.max())
        q = lambda v, p: round(float(torch.quantile(v, p)), 2)
        life = end - start
        print(json.dumps({
            "set": args.set, "waves": int(b.total_tiles), "span_us": round(span, 2),
            "lifetime_us_p10_p50_p90": [q(life, .1), q(life, .5), q(life, .9)],
            "setup_us_p50_p90": [q(issued - start, .5), q(issued - start, .9)],
            "load_wait_us_p50_p90": [q(landed - issued, .5), q(landed - issued, .9)],
            "compute_us_p50_p90": [q(end - landed, .5), q(end - landed, .9)],
            "mean_live_waves": round(float(life.sum()) / span, 1),
            "first_wave_end_us": q(end, 0.0), "start_of_last_wave_us": round(float(start.max()), 2),
            # live waves at 20 instants across the span (ramp at the start, tail at the end)
            "live_waves_timeline": [int(((start <= t) & (end > t)).sum()) for t in
                                    [span * (k + 0.5) / 20 for k in range(20)]],
            "ramp_us_to_90pct_of_peak_live": ramp_time(start, end, span),
            "tail_us_from_90pct_done": round(span - float(torch.quantile(end, 0.9)), 2)}))


def ramp_time(start, end, span):
    """First instant (0.25 us steps) at which the live-wave count reaches 90 % of its peak."""
    ts = torch.arange(0, span, 0.25, dtype=torch.float64)
    live = torch.tensor([int(((start <= t) & (end > t)).sum()) for t in ts.tolist()[:400]])
    peak = int(live.max()) if live.numel() else 0
    idx = (live >= 0.9 * peak).nonzero()
    return round(float(ts[int(idx[0])]), 2) if idx.numel() else None


if __name__ == "__main__":
    main()
