#!/usr/bin/env python3
"""Per-wave timeline of one ragged launch (build variant AWQ_TRACE: every wave records
s_memrealtime at start, after its first tile, at the end, and its tile count).

  make -C awq-converter_amd/csrc variant-trace VFLAGS=-DAWQ_TRACE
  python scripts/trace_waves.py --set opt-125m

Prints the launch span and how the waves fill it: start ramp, first-tile latency, the
end-time distribution (the tail), and the busy fraction sum(end - start) / (waves x span).
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

TICK_NS = 10.0   # s_memrealtime: 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="opt-125m")
    ap.add_argument("--lib", default=os.path.join(ROOT, "awq-converter_amd/awq_quantizer/_lib/variants/libawq_hip_trace.so"))
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    os.environ["AWQ_HIP_LIB"] = args.lib
    from awq_quantizer import _hip
    from awq_quantizer.quantization.batch import PackedBatch
    lib = _hip.load_library()
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
    out = []
    for it in range(3 * args.reps):
        buf.zero_()
        batches[it % args.reps].run()
        torch.cuda.synchronize()
        if it >= args.reps:
            out.append(buf.view(nwaves, 4).cpu())
    assert lib is not None
    res = []
    for tr in out:
        act = tr[:, 3] > 0
        t = tr[act].double()
        t0 = t[:, 0].min()
        start, first, end, n = (t[:, 0] - t0) * TICK_NS / 1e3, (t[:, 1] - t0) * TICK_NS / 1e3, \
            (t[:, 2] - t0) * TICK_NS / 1e3, t[:, 3]
        span = float(end.max())
        q = lambda v, p: float(torch.quantile(v, p))
        busy = float((end - start).sum()) / (len(end) * span)
        res.append({"waves": int(act.sum()), "span_us": round(span, 2),
                    "start_us_p50_p99_max": [round(q(start, .5), 2), round(q(start, .99), 2), round(float(start.max()), 2)],
                    "first_tile_done_us_p10_p50_p90": [round(q(first, .1), 2), round(q(first, .5), 2), round(q(first, .9), 2)],
                    "end_us_p10_p50_p90_p99": [round(q(end, .1), 2), round(q(end, .5), 2), round(q(end, .9), 2), round(q(end, .99), 2)],
                    "tiles_min_max": [int(n.min()), int(n.max())], "busy_fraction": round(busy, 3),
                    "per_tile_us_median": round(q((end - first) / (n - 1).clamp(min=1), .5), 3)})
    for r in res:
        print(json.dumps({"set": args.set, **r}))
    # where the slow waves are: wave w = 4 * block + wid; block b runs on XCD b % 8
    tr = out[-1]
    act = tr[:, 3] > 0
    t = tr.double()
    t0 = t[act, 0].min()
    end = (t[:, 2] - t0) * TICK_NS / 1e3
    w = torch.arange(nwaves)
    blk = w // 4
    xcd = blk % 8
    per_xcd = {int(x): round(float(end[act & (xcd == x)].median()), 1) for x in range(8)}
    slot = (blk // 8) % 256       # block's position within its XCD (~ CU after 8 blocks/CU)
    print(json.dumps({"end_median_by_xcd_us": per_xcd}))
    print(json.dumps({"end_median_by_wid_us": {int(i): round(float(end[act & (w % 4 == i)].median()), 1) for i in range(4)}}))
    # block-level spread inside one XCD and between the 4 waves of a block
    e = end.view(-1, 4)
    print(json.dumps({"within_block_range_us_median": round(float((e.max(1).values - e.min(1).values).median()), 2),
                      "block_end_p10_p50_p90_us": [round(float(torch.quantile(e.max(1).values, q)), 1) for q in (.1, .5, .9)]}))
    bend = e.max(1).values
    order = torch.argsort(bend)
    print(json.dumps({"fastest_blocks": order[:8].tolist(), "slowest_blocks": order[-8:].tolist(),
                      "blocks_per_xcd_in_fastest_quarter": torch.bincount((order[:512] % 8), minlength=8).tolist()}))
    del slot


if __name__ == "__main__":
    main()
