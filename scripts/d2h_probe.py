#!/usr/bin/env python3
"""Why do some of the pipeline's D2H calls block the submitter for 8-11 ms (profiles/round4/
r4f/cli8b.txt, batches 4, 9, 10)?  In a fresh process, after the device warm-up: one fresh
pinned buffer of the CLI's host-ring size, then D2H copies of a given size walking through
it twice; per copy the time inside hipMemcpyAsync (the call) and to completion.  Variants:
the buffer as hipHostMalloc returns it, or first written by the CPU (memset).

  python scripts/d2h_probe.py [--ring-mb 1152] [--copy-mb 64,263] [--touch]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ring-mb", type=int, default=1152)
    ap.add_argument("--copy-mb", default="64,263")
    ap.add_argument("--touch", action="store_true", help="CPU-write the ring before the copies")
    a = ap.parse_args()
    sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
    import torch
    from awq_quantizer import _hip, stream
    lib = _hip.load_library()
    lib.awq_runtime_warmup(0)
    lib.awq_runtime_warmup_wait(0, None)
    hip = ctypes.CDLL("libamdhip64.so")
    s = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
    nbytes = a.ring_mb << 20
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t = time.perf_counter()
    ring = stream.pinned_bytes(nbytes)
    out = {"ring_MB": a.ring_mb, "alloc_ms": round((time.perf_counter() - t) * 1e3, 2), "touch": a.touch}
    if a.touch:
        t = time.perf_counter()
        ctypes.memset(ring.data_ptr(), 0, nbytes)
        out["touch_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    print(json.dumps(out), flush=True)
    for mb in (int(v) for v in a.copy_mb.split(",")):
        n = mb << 20
        for rnd in range(2):
            off = 0
            while off + n <= nbytes:
                t0 = time.perf_counter()
                assert hip.hipMemcpyAsync(ctypes.c_void_p(ring.data_ptr() + off), ctypes.c_void_p(src.data_ptr() + off),
                                          ctypes.c_size_t(n), 2, s) == 0
                t1 = time.perf_counter()
                assert hip.hipStreamSynchronize(s) == 0
                t2 = time.perf_counter()
                print(json.dumps({"copy_MB": mb, "round": rnd, "offset_MB": off >> 20, "call_ms": round((t1 - t0) * 1e3, 2),
                                  "total_ms": round((t2 - t0) * 1e3, 2), "GBs": round(n / (t2 - t0) / 1e9, 1)}), flush=True)
                off += n


if __name__ == "__main__":
    main()
