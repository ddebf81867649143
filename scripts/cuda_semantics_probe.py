"""Where torch's GPU evaluation of the reference's private expressions (awq.py:245 / :282 with
device="cuda") differs from the HIP path's device="cuda" semantics: prints, for the first
mismatching elements of each kind of call, the operands, both results and torch's GPU
intermediate.  Diagnostics only (run on the GPU box)."""
import collections
import json
import os
import sys

import torch
from safetensors.torch import load_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "awq-converter_amd"))
from awq_quantizer.quantization import AWQQuantizer  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
kinds = collections.Counter()
shown = collections.Counter()
for name in ("golden_promote", "golden_promote_int"):
    T = load_file(os.path.join(G, name + ".safetensors"))
    calls = json.load(open(os.path.join(G, name + ".json")))["calls"]
    qs = {}
    for c in calls:
        x, s, z = T[c["x"]], T[c["scale"]], T[c["zero_point"]]
        if "out" not in c or x.dtype in (torch.uint16, torch.uint32, torch.uint64):
            continue
        p = c["params"]
        key = tuple(sorted(p.items()))
        q = qs.setdefault(key, AWQQuantizer(device="cuda", logger_level="ERROR", **p))
        got = getattr(q, c["method"])(x, s, z).cpu()
        xc, sc, zc = x.cuda(), s.cuda(), z.cuda()
        if p["per_channel"] and xc.dim() > 1 and sc.dim() == 1:
            shp = [sc.size(0)] + [1] * (xc.dim() - 1)
            sc, zc = sc.reshape(shp), zc.reshape(shp)
        if c["method"] == "_quantize_tensor":
            inter = xc / sc
            want = torch.clamp(torch.round(inter + zc), q.qmin, q.qmax).cpu()
        else:
            inter = xc - zc
            want = (inter * sc).cpu()
        if got.dtype != want.dtype or got.shape != want.shape:
            kinds[("dtype/shape", c["method"])] += 1
            continue
        gd, wd = got.double(), want.double()
        bad = ~((gd == wd) | (torch.isnan(gd) & torch.isnan(wd)))
        if not bad.any():
            kinds["ok"] += 1
            continue
        k = (c["method"], str(x.dtype), str(s.dtype), str(z.dtype), tuple(s.shape) == (), s.numel() == 1)
        kinds[k] += 1
        if shown[k] < 2:
            shown[k] += 1
            idx = bad.nonzero()[0].tolist()
            xe = x.expand(want.shape) if x.shape != want.shape else x
            print(k, c["x"], c["scale"], "n_bad", int(bad.sum()), "of", bad.numel())
            se = torch.broadcast_to(sc.cpu(), want.shape) if sc.dim() else sc.cpu()
            ze = torch.broadcast_to(zc.cpu(), want.shape) if zc.dim() else zc.cpu()
            ie = torch.broadcast_to(inter.cpu(), want.shape)
            at = lambda t: (t[tuple(idx)] if t.dim() else t).item()
            print("   x", at(xe), "s", at(se), "z", at(ze), "ours", at(got), "torch-gpu", at(want), "inter", at(ie))
for k, v in kinds.most_common():
    print(v, k)
