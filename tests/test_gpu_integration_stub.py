"""the ctypes stub a maintainer of the reference adds
(integration/awq_hip_stub.py), executed as written.

The stub replaces the body of the reference's AWQQuantizer._quantize_per_group
(awq.py:286-374) and keeps its return contract (fp32 [rows, G] scales and zero points,
awq.py:327-328; the small-tensor branch awq.py:297-300).  This test plays the rest of the
reference: `quantize`'s conversions of awq.py:409-416 are restated below (tensor_q and
zero_points to int32, scales to fp16, on the CPU) and applied to the stub's outputs, and
the result must equal the reference's own outputs in tests/golden/ bit for bit.

`self` is this repo's AWQQuantizer, which carries the reference's attributes and private
methods (_calculate_scale_zp / _quantize_tensor, used by the small-tensor branch — in the
real integration that branch is the reference's own code).  Those private methods do not
pin NaN payloads (tests/test_private_methods.py), so small-tensor cases with a NaN scale
compare NaN positions only; every group-path case is exact, NaN bits included.
Needs a gfx950 GPU."""
import importlib.util
import os

import pytest
import torch

import golden_io as gio

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def stub():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    spec = importlib.util.spec_from_file_location("awq_hip_stub", os.path.join(ROOT, "integration", "awq_hip_stub.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from awq_quantizer import _hip
    mod.load(_hip.LIB_PATH)
    return mod


def _reference_quantize(stub, q, x):
    """awq.py:376-433 with the stub in place of _quantize_per_group: the dict conversions
    of awq.py:409-416, restated."""
    tq, s, z = stub.quantize_per_group(q, x)
    return {"tensor_q": tq.cpu().to(torch.int32), "scales": s.cpu().to(torch.float16),
            "zero_points": z.cpu().to(torch.int32)}


def _q(p):
    from awq_quantizer.quantization import AWQQuantizer
    return AWQQuantizer(device="cpu", logger_level="ERROR", **p)


def _check(res, T, name, small_nan_ok):
    assert torch.equal(res["tensor_q"], T[name + ".tensor_q"]), "tensor_q"
    assert torch.equal(res["zero_points"], T[name + ".zero_points"]), "zero_points"
    want = T[name + ".scales"]
    if small_nan_ok:
        assert torch.equal(torch.isnan(res["scales"]), torch.isnan(want))
        keep = ~torch.isnan(want)
        assert gio.same_bits(res["scales"][keep], want[keep])
    else:
        assert gio.same_bits(res["scales"], want), "scales"


@pytest.mark.parametrize("case", gio.ok_cases(), ids=lambda c: c["name"])
def test_stub_matches_reference_golden(stub, case):
    x = gio.case_input(case)
    p = case["params"]
    res = _reference_quantize(stub, _q(p), x)
    small = x.numel() < p["group_size"]
    _check(res, gio.tensors(), case["name"], small)
    if not small:
        tq, s, z = stub.quantize_per_group(_q(p), x)
        assert s.dtype == torch.float32 and z.dtype == torch.float32 and tq.dtype == torch.int32   # awq.py:327-329
        assert s.device.type == "cpu"


@pytest.mark.parametrize("case", gio.nan_cases(), ids=lambda c: c["name"])
def test_stub_matches_reference_nan_cases(stub, case):
    x = gio.nan_case_input(case)
    p = case["params"]
    res = _reference_quantize(stub, _q(p), x)
    _check(res, gio.nan_tensors(), case["name"], x.numel() < p["group_size"])


def test_stub_fp32_scale_values_are_the_dtype_values(stub):
    """The stub's fp32 scales are the input dtype's own scale values (awq.py:352), not their
    fp16 rounding: fp32 weights keep fp32-valued scales (24-bit significands)."""
    from oracle import awq_oracle as orc
    g = torch.Generator().manual_seed(3)
    x = torch.randn(64, 512, generator=g) * 0.02
    q = _q(dict(bits=4, group_size=128, symmetric=False))
    _, s, _ = stub.quantize_per_group(q, x)
    want, _ = orc.group_params(x, 64, 512, 128, 4, False)
    assert torch.equal(s, want.to(torch.float32))
    assert not torch.equal(s, s.to(torch.float16).to(torch.float32))   # bf16 values are not fp16 values
