"""Helpers to read the golden fixtures written by tests/golden/make_golden.py."""
import json
import os

import torch
from safetensors.torch import load_file

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_DT = {"torch.bfloat16": torch.bfloat16, "torch.float16": torch.float16,
       "torch.float32": torch.float32, "torch.float64": torch.float64,
       "bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32, "f64": torch.float64}

_cache = {}


def manifest():
    if "m" not in _cache:
        with open(os.path.join(GOLDEN_DIR, "golden_manifest.json")) as f:
            _cache["m"] = json.load(f)
    return _cache["m"]


def tensors():
    if "t" not in _cache:
        _cache["t"] = load_file(os.path.join(GOLDEN_DIR, "golden_small.safetensors"))
    return _cache["t"]


def case_input(case):
    t = tensors()[case["input"]]
    dt = _DT[case["dtype"]]
    if dt == torch.bfloat16:
        t = t.view(torch.bfloat16)
    return t.reshape(case["shape"])


def ok_cases():
    return [c for c in manifest()["cases"] if c.get("ok") and "input" in c]


def hashed_input(rec):
    g = torch.Generator().manual_seed(rec["seed"])
    x = torch.randn(*rec["shape"], generator=g, dtype=torch.float32) * rec["scale"]
    return x.to(_DT[rec["dtype"]])


def sha(t):
    import hashlib
    t = t.contiguous().cpu()
    if t.dtype == torch.bfloat16:
        t = t.view(torch.int16)
    return hashlib.sha256(t.numpy().tobytes()).hexdigest()


def same_bits_nan_eq(a, b):
    """Bit equality, except that any NaN matches any NaN (NaN payload/sign is not pinned)."""
    a, b = a.contiguous(), b.contiguous()
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    if a.is_floating_point():
        an, bn = torch.isnan(a), torch.isnan(b)
        if not torch.equal(an, bn):
            return False
        ia = a.view(torch.int16 if a.element_size() == 2 else (torch.int32 if a.element_size() == 4 else torch.int64))
        ib = b.view(ia.dtype)
        return bool(torch.equal(ia[~an], ib[~bn]))
    return bool(torch.equal(a, b))
