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


def same_bits(a, b):
    """Exact bit equality of two tensors (NaN payloads and signs included)."""
    a, b = a.contiguous().cpu(), b.contiguous().cpu()
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    if a.is_floating_point():
        it = {2: torch.int16, 4: torch.int32, 8: torch.int64}[a.element_size()]
        return bool(torch.equal(a.view(it), b.view(it)))
    return bool(torch.equal(a, b))


# ---- NaN-origin fixtures (make_golden.py --nan) ----
def nan_manifest():
    if "nm" not in _cache:
        with open(os.path.join(GOLDEN_DIR, "golden_nan.json")) as f:
            _cache["nm"] = json.load(f)
    return _cache["nm"]


def nan_tensors():
    if "nt" not in _cache:
        _cache["nt"] = load_file(os.path.join(GOLDEN_DIR, "golden_nan.safetensors"))
    return _cache["nt"]


def nan_cases():
    return [c for c in nan_manifest()["cases"] if c.get("ok")]


def nan_case_input(case):
    t = nan_tensors()[case["input"]]
    if _DT[case["dtype"]] == torch.bfloat16:
        t = t.view(torch.bfloat16)
    return t.reshape(case["shape"])
