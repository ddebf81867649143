#!/usr/bin/env python3
"""Does starting the device warm-up before `import torch` (awq_quantizer/_early.py) slow the
import down?  Fresh processes, alternating variants:
  torch        import torch; then torch.cuda.init + first allocation
  early        _early.start; import torch; then the warm-up's join; then torch.cuda.init +
               first allocation
  early_late   import torch; then _early.start + join (the warm-up after the import)
per run: seconds of each step, from inside the child.

  python scripts/early_probe.py [--runs 3]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, json, sys, time
t0 = time.time()
variant = sys.argv[1]
out = {"variant": variant}
from awq_quantizer import _early
if variant == "early":
    _early.start([])
    out["start_s"] = round(time.time() - t0, 4)
t = time.time()
import torch
out["import_torch_s"] = round(time.time() - t, 4)
if variant in ("early", "early_late"):
    t = time.time()
    if variant == "early_late":
        _early.start([])
    lib = ctypes.CDLL(_early.LIB_PATH)
    secs = ctypes.c_double(0)
    lib.awq_runtime_warmup_wait(0, ctypes.byref(secs))
    out["warmup_join_s"] = round(time.time() - t, 4)
    out["warmup_own_s"] = round(secs.value, 4)
t = time.time()
torch.cuda.init()
torch.empty(1, device="cuda")
torch.cuda.synchronize()
out["torch_cuda_init_s"] = round(time.time() - t, 4)
out["total_s"] = round(time.time() - t0, 4)
print("RESULT " + json.dumps(out), flush=True)
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--variants", default="torch,early,early_late")
    a = ap.parse_args()
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "awq-converter_amd"), ROOT]))
    for r in range(a.runs):
        for v in a.variants.split(","):
            t = time.time()
            p = subprocess.run([sys.executable, "-c", CHILD, v], capture_output=True, text=True, timeout=300, env=env)
            wall = time.time() - t
            res = [ln[7:] for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
            if p.returncode or not res:
                print(json.dumps({"variant": v, "rc": p.returncode, "err": p.stderr[-800:]}), flush=True)
                sys.exit(1)
            d = json.loads(res[0])
            d.update({"run": r, "process_wall_s": round(wall, 3)})
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
