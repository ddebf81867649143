#!/usr/bin/env python3
"""Cost of page-locked host memory in a FRESH process (the CLI's first-run setup), per method
and size, and the D2H rate into it:
  torch     torch.empty(pin_memory=True)   (torch's caching host allocator: power-of-two sizes)
  hostmalloc hipHostMalloc(exact size)
  register  anonymous mmap, pages touched by T threads, then hipHostRegister
Each method in its own child process (a fresh heap), one JSON line per (method, size).

  python scripts/pin_probe.py --sizes-mb 256,1024,4096 --threads 8
"""
import argparse
import ctypes
import json
import mmap
import os
import subprocess
import sys
import time


def child(method, mb, threads):
    import torch
    from concurrent.futures import ThreadPoolExecutor
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    src = torch.empty(mb << 20, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    nbytes = mb << 20
    t0 = time.perf_counter()
    keep = None
    if method == "twoalloc":
        # is the first D2H's extra cost per process (copy machinery) or per allocation?
        hip = _hip = ctypes.CDLL("libamdhip64.so")
        bufs = []
        for _ in range(2):
            p = ctypes.c_void_p()
            assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes), 0) == 0
            bufs.append(torch.frombuffer((ctypes.c_char * nbytes).from_address(p.value), dtype=torch.uint8))
        out = {"method": method, "MB": mb}
        for k, b in enumerate(bufs + bufs):
            torch.cuda.synchronize()
            t = time.perf_counter()
            b.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            out[f"d2h_{k}_GBs"] = round(nbytes / (time.perf_counter() - t) / 1e9, 1)
        print(json.dumps(out), flush=True)
        return
    if method == "torch":
        h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        ptr = h.data_ptr()
        keep = h
    elif method == "hostmalloc":
        p = ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes), 0) == 0
        ptr = p.value
    else:
        m = mmap.mmap(-1, nbytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        buf = (ctypes.c_char * nbytes).from_buffer(m)
        base = ctypes.addressof(buf)
        step = -(-nbytes // threads)

        def touch(k):
            lo, hi = k * step, min(nbytes, (k + 1) * step)
            if hi > lo:
                ctypes.memset(base + lo, 0, hi - lo)
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(touch, range(threads)))
        t_touch = time.perf_counter() - t0
        assert hip.hipHostRegister(ctypes.c_void_p(base), ctypes.c_size_t(nbytes), 0) == 0
        ptr = base
        keep = (m, buf)
    t_alloc = time.perf_counter() - t0
    hview = torch.frombuffer((ctypes.c_char * nbytes).from_address(ptr), dtype=torch.uint8)
    rates = []
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        hview.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        rates.append(nbytes / (time.perf_counter() - t) / 1e9)
    out = {"method": method, "MB": mb, "threads": threads, "alloc_s": round(t_alloc, 4),
           "alloc_GBs": round(nbytes / t_alloc / 1e9, 2), "d2h_GBs_first": round(rates[0], 1),
           "d2h_GBs_best": round(max(rates), 1)}
    if method == "register":
        out["touch_s"] = round(t_touch, 4)
    print(json.dumps(out), flush=True)
    del keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="256,1024,4096")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--methods", default="torch,hostmalloc,register")
    ap.add_argument("--child", nargs=3)
    a = ap.parse_args()
    if a.child:
        child(a.child[0], int(a.child[1]), int(a.child[2]))
        return
    for mb in (int(v) for v in a.sizes_mb.split(",")):
        for m in a.methods.split(","):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", m, str(mb), str(a.threads)],
                               capture_output=True, text=True, timeout=300)
            sys.stdout.write(r.stdout)
            if r.returncode:
                print(json.dumps({"method": m, "MB": mb, "rc": r.returncode, "err": r.stderr[-400:]}))
            sys.stdout.flush()


if __name__ == "__main__":
    main()
