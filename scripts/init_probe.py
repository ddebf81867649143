#!/usr/bin/env python3
"""Per-process first-use costs the CLI pays before its pipeline runs ("CLI, fresh
process"): each step timed once in a FRESH child process, in the order the CLI meets them,
most steps twice so the first-use part stands out.

  python scripts/init_probe.py [--runs 2]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    out = []
    t = [time.perf_counter()]

    def mark(name):
        now = time.perf_counter()
        out.append((name, round((now - t[0]) * 1e3, 2)))
        t[0] = now

    import torch
    mark("import torch")
    torch.cuda.init()
    torch.empty(1, device="cuda")
    torch.cuda.synchronize()
    mark("cuda init + first alloc")
    sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
    from awq_quantizer import _hip, stream
    lib = _hip.load_library()
    mark("load libawq_hip.so")
    hip = ctypes.CDLL("libamdhip64.so")
    name = ctypes.create_string_buffer(256)
    assert hip.hipDeviceGetName(name, 256, 0) == 0
    mark("hipDeviceGetName")
    torch.cuda.mem_get_info(0)
    mark("mem_get_info #1")
    torch.cuda.mem_get_info(0)
    mark("mem_get_info #2")
    tname = torch.cuda.get_device_name(0)
    mark("get_device_name")
    out.append(("names equal", name.value.decode() == tname))
    raw = []
    for k in range(2):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
        raw.append(s)
        mark(f"hipStreamCreateWithFlags #{k + 1}")
    ts = [torch.cuda.Stream() for _ in range(1)]
    mark("torch.cuda.Stream #1")
    ts.append(torch.cuda.Stream())
    mark("torch.cuda.Stream #2")
    d = torch.empty(768 << 20, dtype=torch.uint8, device="cuda")
    mark("device alloc 768 MiB")
    h = stream.pinned_bytes(800 << 20)
    mark("hipHostMalloc 800 MiB")
    s = raw[0]
    for n, tag in ((256, "256 B"), (64 << 10, "64 KiB"), (1 << 20, "1 MiB"), (8 << 20, "8 MiB"),
                   (8 << 20, "8 MiB again"), (256 << 20, "256 MiB")):
        assert hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(h.data_ptr()), ctypes.c_size_t(n), 1, s) == 0
        assert hip.hipStreamSynchronize(s) == 0
        mark(f"H2D {tag}")
    s = raw[1]
    for n, tag in ((256, "256 B"), (8 << 20, "8 MiB"), (8 << 20, "8 MiB again"), (256 << 20, "256 MiB")):
        assert hip.hipMemcpyAsync(ctypes.c_void_p(h.data_ptr()), ctypes.c_void_p(d.data_ptr()), ctypes.c_size_t(n), 2, s) == 0
        assert hip.hipStreamSynchronize(s) == 0
        mark(f"D2H {tag}")
    for k in range(2):
        rc = lib.awq_stream_copy(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(d.data_ptr() + (256 << 20)),
                                 ctypes.c_int64(1 << 20), s)
        assert rc == 0, _hip.last_error()
        assert hip.hipStreamSynchronize(s) == 0
        mark(f"first kernel of libawq_hip #{k + 1}")
    # pinned allocations, serial vs two threads (does the driver serialise them?)
    from concurrent.futures import ThreadPoolExecutor
    keep = [stream.pinned_bytes(400 << 20), stream.pinned_bytes(400 << 20)]
    mark("hipHostMalloc 2 x 400 MiB serial")
    with ThreadPoolExecutor(2) as ex:
        keep += list(ex.map(lambda _: stream.pinned_bytes(400 << 20), range(2)))
    mark("hipHostMalloc 2 x 400 MiB on two threads")
    del keep
    print("RESULT " + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child()
        return
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "awq-converter_amd"), ROOT]))
    for r in range(a.runs):
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], capture_output=True, text=True,
                           timeout=300, env=env)
        res = [ln[7:] for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
        if p.returncode or not res:
            print(json.dumps({"run": r, "rc": p.returncode, "err": p.stderr[-1500:]}), flush=True)
            sys.exit(1)
        print(json.dumps({"run": r, "ms": dict(json.loads(res[0]))}), flush=True)   # ("names equal": bool)


if __name__ == "__main__":
    main()
