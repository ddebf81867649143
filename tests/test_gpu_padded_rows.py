"""Padded rows on the streaming kernel: K % group_size != 0 with K % 8 == 0 (e.g. Falcon-7B's
hidden size 4544 at group size 128, 1-D tensors like (5000,)).  The reference zero-pads each
row's tail group for its min/max (awq.py:337-339) and keeps only the K real elements in
tensor_q; the kernel tiles such tensors by rows and lets the buffer range check supply the
padding zeros (include/awq_hip.h, awq_internal.h "row tiles").  Bit-exact against the oracle.
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


def rand(shape, seed, scale=0.02, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


def shapes_for(gs):
    return [(7, 3 * gs + 8), (5, 5 * gs + gs // 2), (10, gs - 8), (3, 40 * gs + 24), (3 * gs + 8,),
            (5000,), (2, 3, 1512), (33, 17 * gs + 64 % gs + 8)]


def check(x, gs, sym, bits, dq=True):
    from awq_quantizer import _hip
    rows = 1 if x.dim() <= 1 else x.shape[0]
    K = x.numel() // rows
    assert K % gs and _hip.ragged_eligible(x.dtype, rows, K, gs), (tuple(x.shape), gs)
    ref = orc.quantize(x, bits=bits, group_size=gs, symmetric=sym)
    q = Q(bits=bits, group_size=gs, symmetric=sym)
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
    pk = q.quantize_packed(x)
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"].reshape(rows, K), bits, q.qmin))
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], bits, q.qmin))
    assert gio.same_bits(pk["scales"].cpu(), ref["scales"])
    if dq:   # (packed fields cannot carry the reference's INT32_MIN for NaN elements)
        assert gio.same_bits(q.dequantize_packed(pk).cpu(), orc.dequantize(ref))


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32], ids=["bf16", "f16", "f32"])
@pytest.mark.parametrize("gs", [32, 64, 128, 256])
def test_padded_rows_vs_oracle(gs, dtype, sym, bits):
    for i, shape in enumerate(shapes_for(gs)):
        shape = tuple(s for s in shape)
        K = shape[-1] if len(shape) == 1 else int(torch.Size(shape[1:]).numel())
        if K % gs == 0:
            continue
        check(rand(shape, 300 * gs + 7 * i + 2 * sym + bits, 0.02, dtype), gs, sym, bits)


@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def test_padded_rows_special_values(dtype, sym):
    """The tail group's padding zeros take part in min/max: an all-positive or all-negative
    row tail gets 0 as its min / max, exactly like the reference's F.pad."""
    x = rand((12, 4544), 77, 1.0, dtype).float()
    x[0, 4480:] = x[0, 4480:].abs() + 3.0          # tail group all positive: min = padding 0
    x[1, 4480:] = -(x[1, 4480:].abs() + 3.0)       # all negative: max = padding 0
    x[2, 4480:] = float("nan")
    x[3, 4490] = float("inf")
    x[4, :128] = 0.0
    x[5, 4480:] = 1e-6
    check(x.to(dtype), 128, sym, 4, dq=False)


@pytest.mark.parametrize("gs", [64, 128])
def test_padded_rows_ragged_mixed(gs):
    """One ragged launch mixing padded-row tensors with flat-tiled ones."""
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device(DEV, 0)
    shapes = [(4544,), (64, 4544), (300, 2 * gs), (7, 3 * gs + 8), (5000,), (40, 12 * gs), (1, 8 + gs)]
    inputs = {f"t{i}": rand(s, 900 + i).to(dev) for i, s in enumerate(shapes)}
    for bits in (4, 8):
        b = PackedBatch(inputs, bits=bits, symmetric=False, parity=True, group_size=gs)
        b.run()
        torch.cuda.synchronize()
        for name, res in b.results().items():
            x = inputs[name].cpu()
            rows = 1 if x.dim() == 1 else x.shape[0]
            ref = orc.quantize(x, bits=bits, group_size=gs, symmetric=False)
            assert torch.equal(res["tensor_q"].cpu(), ref["tensor_q"]), name
            assert torch.equal(res["zero_points"].cpu(), ref["zero_points"].reshape(rows, -1)), name
            assert gio.same_bits(res["scales"].cpu(), ref["scales"].reshape(rows, -1)), name
            assert torch.equal(res["qweight"].cpu(), orc.pack_rows(ref["tensor_q"].reshape(rows, -1), bits, 0)), name
            assert torch.equal(res["qzeros"].cpu(), orc.pack_rows(ref["zero_points"].reshape(rows, -1), bits, 0)), name


@pytest.mark.parametrize("sym", [False, True])
def test_padded_rows_clip_search(sym):
    x = rand((24, 4544), 4545 + sym, 1.0)
    q = Q(bits=4, group_size=128, symmetric=sym, scale_method="search")
    ref = orc.quantize(x, bits=4, group_size=128, symmetric=sym, search=(20, 10))
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
