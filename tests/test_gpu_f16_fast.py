"""fp16 inputs on the streaming kernel (FmtF16 in csrc/awq_fast.hip) against the oracle.

The reference computes an fp16 tensor's ops in fp16 (torch CPU: fp32 math, RNE to fp16
per op).  The kernel forms x / s as the plain x * RN(1/s) in tiles whose scales are all
< 14 (exhaustively exact there: test_oracle_golden.py::
test_f16_plain_product_small_scales_exhaustive) and with a Markstein-corrected quotient
otherwise (exact over all fp16 pairs: test_f16_markstein_division_exhaustive),
the scale and zero point with IEEE divisions, and routes groups whose scale is 0 (the fp16
clamp min RN_f16(1e-10) is 0: constant groups), inf or NaN through an exact per-element
division.  Bar: bit-exact int32 values, fp16 scales, packed words.
"""
import pytest
import torch

import golden_io as gio
from oracle import awq_oracle as orc

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer import _hip
    _hip.require_device(torch.device("cuda", 0))


def Q(**kw):
    from awq_quantizer.quantization import AWQQuantizer
    kw.setdefault("device", DEV)
    return AWQQuantizer(logger_level="ERROR", **kw)


def rand16(shape, seed, scale):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.float16)


def check(x, bits, sym):
    ref = orc.quantize(x, bits=bits, group_size=128, symmetric=sym)
    q = Q(bits=bits, symmetric=sym)
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
    pk = q.quantize_packed(x)
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], bits, q.qmin))
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], bits, q.qmin))
    assert gio.same_bits(pk["scales"].cpu(), ref["scales"])


def test_f16_takes_the_streaming_kernel():
    from awq_quantizer import _hip
    assert _hip.ragged_eligible(torch.float16, 1024, 4096, 128)
    assert not _hip.ragged_eligible(torch.float64, 1024, 4096, 128)


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("shape,scale", [((1024, 4096), 0.02), ((4096, 768), 1.0), ((768,), 0.5), ((7, 1792), 3e-3),
                                         ((33, 11 * 128), 300.0), ((77, 768), 2e-5), ((3, 896), 1e4)], ids=str)
def test_f16_fast_vs_oracle(shape, scale, sym, bits):
    check(rand16(shape, hash((shape, sym, bits)) & 0xFFFF, scale), bits, sym)


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [False, True])
def test_f16_special_values(sym, bits):
    """NaN, +-inf, 65504, subnormals, signed zeros, and constant groups (scale 0)."""
    x = rand16((64, 1024), 11 + bits + sym, 1.0).float()
    flat = x.view(-1)
    g = torch.Generator().manual_seed(3)
    idx = torch.randperm(flat.numel(), generator=g)[:400]
    kinds = [float("nan"), float("inf"), float("-inf"), 65504.0, -65504.0, 6e-8, -6e-8, 0.0, -0.0, 1e-5]
    for i, j in enumerate(idx.tolist()):
        flat[j] = kinds[i % len(kinds)]
    x[0, :128] = 0.0              # all zero: s = 0 -> x / 0 = NaN -> INT_MIN
    x[1, :128] = 1.0              # constant positive: s = 0, 1 / 0 = inf
    x[2, 128:256] = -2.5          # constant negative
    x[3, :128] = 6e-8             # constant subnormal
    x[4, 256:384] = torch.linspace(-1e-7, 1e-7, 128)   # subnormal range: tiny scale
    check(x.to(torch.float16), bits, sym)


@pytest.mark.parametrize("bits", [4, 8])
def test_f16_every_scale_value(bits):
    """Groups [m, 0, 0, ...] for every positive finite fp16 m: every scale RN(m / (2^b-1))
    and every quotient m / s the kernel can form for such a group, against the oracle."""
    m = torch.arange(1, 0x7C00, dtype=torch.int32).to(torch.int16).view(torch.float16)
    x = torch.zeros(m.numel(), 128, dtype=torch.float16)
    x[:, 0] = m
    x[:, 1] = m * 0.37
    check(x, bits, False)


def test_f16_ragged_and_model_packed():
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device(DEV, 0)
    shapes = [(768,), (768, 768), (3072, 768), (9, 1792), (128,)]
    inputs = {f"t{i}": rand16(s, 50 + i, 0.02).to(dev) for i, s in enumerate(shapes)}
    b = PackedBatch(inputs, bits=4, symmetric=False, parity=True)
    b.run()
    torch.cuda.synchronize()
    for name, res in b.results().items():
        ref = orc.quantize(inputs[name].cpu(), bits=4, group_size=128, symmetric=False)
        assert torch.equal(res["tensor_q"].cpu(), ref["tensor_q"]), name
        assert torch.equal(res["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], 4, 0)), name
        assert gio.same_bits(res["scales"].cpu(), ref["scales"]), name
    # mixed dtypes: one ragged launch per dtype
    mixed = {"a": rand16((256, 512), 1, 0.02), "b": rand16((512,), 2, 0.02).to(torch.bfloat16)}
    out = Q(bits=4, symmetric=False).quantize_model_packed(mixed)
    for name, t in mixed.items():
        ref = orc.quantize(t, bits=4, group_size=128, symmetric=False)
        rows = 1 if t.dim() == 1 else t.shape[0]
        assert torch.equal(out[name]["qweight"].cpu(), orc.pack_rows(ref["tensor_q"].reshape(rows, -1), 4, 0)), name
    with pytest.raises(ValueError, match="one dtype"):
        PackedBatch({"a": mixed["a"].to(dev), "b": mixed["b"].to(dev)})


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("bound", [100.0, 1.0, 1e-3])
def test_f16_plain_quotient_tiles_random_bits(bits, sym, bound):
    """Every fp16 bit pattern of magnitude < bound (subnormals, zeros of both signs): all
    scales < 14, so every tile takes the plain-product quotient."""
    g = torch.Generator().manual_seed(int(bound * 1000) + bits)
    bitsv = torch.randint(0, 0x7C00, (512 * 128,), generator=g, dtype=torch.int32)
    sign = torch.randint(0, 2, bitsv.shape, generator=g, dtype=torch.int32) << 15
    x = (bitsv | sign).to(torch.int16).view(torch.float16).reshape(512, 128)
    x = torch.where(x.abs() < bound, x, x * 0)
    check(x, bits, sym)


@pytest.mark.parametrize("bits", [4, 8])
def test_f16_mixed_plain_and_markstein_tiles(bits):
    """Large-range groups (scale >= 14) next to ordinary ones: tiles of both kinds."""
    x = rand16((256, 1024), 11, 0.05).float()
    x[::7, :128] *= 30000.0 / x[::7, :128].abs().max()
    check(x.to(torch.float16), bits, False)
