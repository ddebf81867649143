"""NaN bits on the HIP path, against the reference's own NaN-origin outputs
(tests/golden/golden_nan.*, make_golden.py --nan) — no NaN latitude anywhere.

The fp16 bits of a NaN scale depend on the input dtype, on whether the group holds a NaN
or got it from inf - inf, on one-element groups and on the small-tensor path
(include/awq_hip.h, oracle_nan_scale_f16); the fp32 dequantize output of a NaN product
depends on its position in its group (the reference's fp16 -> fp32 copy).  Every kernel
(streaming, row-segment, generic fp64 span and register span, the clip search, the ragged
launch, packed dequantize) is driven through these cases.  Needs a gfx950 GPU.
"""
import pytest
import torch

import golden_io as gio
from oracle import awq_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer import _hip
    _hip.require_device(torch.device("cuda", 0))


def Q(**kw):
    from awq_quantizer.quantization import AWQQuantizer
    kw.setdefault("device", "cuda")
    return AWQQuantizer(logger_level="ERROR", **kw)


@pytest.mark.parametrize("case", gio.nan_cases(), ids=lambda c: c["name"])
def test_nan_case_exact(case):
    x = gio.nan_case_input(case)
    p = case["params"]
    q = Q(**p)
    res = q.quantize(x)
    T = gio.nan_tensors()
    name = case["name"]
    assert torch.equal(res["tensor_q"], T[name + ".tensor_q"]), "tensor_q"
    assert torch.equal(res["zero_points"], T[name + ".zero_points"]), "zero_points"
    assert gio.same_bits(res["scales"], T[name + ".scales"]), "scales"
    if name + ".dq" in T:
        assert gio.same_bits(q.dequantize(res), T[name + ".dq"]), "dequantize"


def _group_cases():
    return [c for c in gio.nan_cases() if gio.nan_tensors()[c["name"] + ".scales"].dim() == 2]


@pytest.mark.parametrize("case", _group_cases(), ids=lambda c: c["name"])
def test_nan_case_packed(case):
    """quantize_packed: the same scales, qweight = the packing of the reference's tensor_q;
    dequantize_packed = the reference's dequantize of the packed values bit for bit."""
    x = gio.nan_case_input(case)
    p = case["params"]
    q = Q(**p)
    pk = q.quantize_packed(x)
    T = gio.nan_tensors()
    name = case["name"]
    rows = pk["scales"].shape[0]
    tq = T[name + ".tensor_q"].reshape(rows, -1)
    qmin = -(2 ** (p["bits"] - 1)) if p["symmetric"] else 0
    assert gio.same_bits(pk["scales"].cpu(), T[name + ".scales"]), "scales"
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(tq, p["bits"], qmin)), "qweight"
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(T[name + ".zero_points"], p["bits"], qmin)), "qzeros"
    # dequantize_packed = the reference's dequantize of the values the packed words hold (a
    # NaN element's INT32_MIN packs to (INT32_MIN - qmin) & mask, so those are not the
    # reference's tensor_q: compare with the oracle on the unpacked values)
    K = tq.shape[1]
    G = pk["scales"].shape[1]
    unp = {"tensor_q": _unpack(pk["qweight"].cpu(), K, p["bits"], qmin).reshape(T[name + ".tensor_q"].shape),
           "zero_points": _unpack(pk["qzeros"].cpu(), G, p["bits"], qmin), "scales": pk["scales"].cpu(),
           "group_size": torch.tensor(p["group_size"], dtype=torch.int32)}
    want = orc.dequantize(unp)
    assert gio.same_bits(q.dequantize_packed(pk).cpu().reshape(want.shape), want)


def _unpack(words, n, bits, qmin):
    """[rows, ceil(n*bits/32)] packed words -> int32 [rows, n] values (field + qmin)."""
    per = 32 // bits
    w = words.to(torch.int64) & 0xFFFFFFFF
    sh = torch.arange(per, dtype=torch.int64) * bits
    f = (w[:, :, None] >> sh) & ((1 << bits) - 1)
    return (f.reshape(words.shape[0], -1)[:, :n] + qmin).to(torch.int32)


@pytest.mark.parametrize("case", [c for c in gio.nan_cases() if c["params"]["group_size"] <= 512],
                         ids=lambda c: c["name"])
def test_nan_case_search_keeps_rtn_bits(case):
    """scale_method="search": NaN / inf groups keep the RTN result, NaN bits included; every
    group equals the oracle's search."""
    x = gio.nan_case_input(case)
    p = case["params"]
    q = Q(scale_method="search", search_grid=10, search_max_shrink=0.5, **p)
    res = q.quantize(x)
    ref = orc.quantize(x, bits=p["bits"], group_size=p["group_size"], symmetric=p["symmetric"],
                       per_channel=p["per_channel"], search=(10, 5))
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
    T = gio.nan_tensors()
    s = T[case["name"] + ".scales"]
    nan = torch.isnan(s)
    assert gio.same_bits(res["scales"][nan], s[nan])          # NaN groups: the reference's RTN bits


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
def test_nan_ragged_launch(dt):
    """The one-launch model path (ragged streaming kernel) gives the same NaN bits."""
    T = gio.nan_tensors()
    cases = [c for c in gio.nan_cases() if c["dtype"] == str(dt) and c["params"]["group_size"] == 128
             and c["params"]["bits"] == 4 and not c["params"]["symmetric"] and len(c["shape"]) == 2
             and c["shape"][1] % 128 == 0]
    assert cases
    q = Q(bits=4, group_size=128, symmetric=False)
    tensors = {c["name"]: gio.nan_case_input(c) for c in cases}
    out = q.quantize_model_device(tensors, packed=False)
    for c in cases:
        r = out[c["name"]]
        assert torch.equal(r["tensor_q"].cpu(), T[c["name"] + ".tensor_q"])
        assert gio.same_bits(r["scales"].cpu(), T[c["name"] + ".scales"]), c["name"]


@pytest.mark.parametrize("dt", [torch.float16, torch.float32, torch.float64])
@pytest.mark.parametrize("sym", [False, True])
def test_nan_scale_rule_large_random(dt, sym):
    """Large tensors (every kernel's tiling): NaNs / infs scattered over 4096 x 4096 at group
    sizes 128 (streaming / fp64 register span), 100 (row-segment / fp64 strided span) and
    1024 (generic) — scales, tensor_q and dequantize equal the oracle's bit for bit."""
    g = torch.Generator().manual_seed(91)
    x = torch.randn(512, 4096, generator=g).to(dt)
    idx = torch.randint(0, x.numel(), (300,), generator=g)
    x.view(-1)[idx[:100]] = float("nan")
    x.view(-1)[idx[100:200]] = float("inf")
    x.view(-1)[idx[200:]] = float("-inf")
    x[7, 0:128] = float("inf")                      # inf - inf groups
    x[9, 128:256] = float("-inf")
    for gs in (128, 100, 1024):
        q = Q(bits=4, group_size=gs, symmetric=sym)
        res = q.quantize(x)
        ref = orc.quantize(x, bits=4, group_size=gs, symmetric=sym)
        assert torch.equal(res["tensor_q"], ref["tensor_q"]), gs
        assert gio.same_bits(res["scales"], ref["scales"]), gs
        assert gio.same_bits(q.dequantize(res), orc.dequantize(ref)), gs
