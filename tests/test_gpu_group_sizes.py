"""Streaming kernel at group sizes 32, 64 and 256 (bf16 / fp16; K % group_size == 0):
bit-exact against the oracle like the group-size-128 path (tests/test_gpu_parity.py).

The reference computes every group size with the same per-group arithmetic
(awq.py:286-374); only the tiling changes on the GPU (2048-element tiles of 2048 / gs
groups, gs / 8 lanes per group, include/awq_hip.h awq_plan_ragged).  Shapes cover byte
tiles (G even or 8-bit), word tiles (4-bit, G odd: whole rows or whole qzeros words per
tile), partial last tiles, 1-D and 3-D tensors, and groups spanning the 16-lane DPP rows
(gs 256).
"""
import pytest
import torch

import golden_io as gio
from oracle import awq_oracle as orc

pytestmark = pytest.mark.gpu

DEV = "cuda"
GROUP_SIZES = [32, 64, 256]


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
    """K multiples of gs with G = 1, 2, 3 (odd: word tiles), 5, 8, 9, 32, 33, ... and row
    counts that leave partial last tiles."""
    return [(64, 32 * gs), (7, 3 * gs), (11, gs), (5, 5 * gs), (3, 9 * gs), (33, 8 * gs), (2, 33 * gs),
            (6 * gs,), (2, 3, 2 * gs), (1, 64 * gs), (129, 2 * gs)]


def check(x, gs, sym, bits):
    ref = orc.quantize(x, bits=bits, group_size=gs, symmetric=sym)
    q = Q(bits=bits, group_size=gs, symmetric=sym)
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
    pk = q.quantize_packed(x)
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], bits, q.qmin))
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], bits, q.qmin))
    assert gio.same_bits(pk["scales"].cpu(), ref["scales"])
    return q, pk, ref


def test_group_sizes_take_the_streaming_kernel():
    from awq_quantizer import _hip
    for gs in GROUP_SIZES + [128]:
        assert _hip.ragged_eligible(torch.bfloat16, 7, 3 * gs, gs)
        assert _hip.ragged_eligible(torch.float16, 7, 3 * gs, gs)
        assert _hip.ragged_eligible(torch.float32, 7, 3 * gs, gs)
        assert not _hip.ragged_eligible(torch.float64, 7, 3 * gs, gs)


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("gs", GROUP_SIZES)
def test_group_size_vs_oracle(gs, dtype, sym, bits):
    for i, shape in enumerate(shapes_for(gs)):
        x = rand(shape, 1000 * gs + 10 * i + 2 * sym + bits, 0.02, dtype)
        check(x, gs, sym, bits)


def special(shape, gs, seed, dtype):
    x = rand(shape, seed, 1.0, torch.float32)
    flat = x.view(-1)
    g = torch.Generator().manual_seed(seed + 1)
    idx = torch.randperm(flat.numel(), generator=g)[: max(8, flat.numel() // 300)]
    big = 3e38 if dtype == torch.bfloat16 else 6e4
    tiny = 1e-39 if dtype == torch.bfloat16 else 1e-7
    kinds = [float("nan"), float("inf"), float("-inf"), big, -big, tiny, 0.0, -0.0]
    for i, j in enumerate(idx.tolist()):
        flat[j] = kinds[i % len(kinds)]
    x[0, :gs] = 0.0                              # all-zero group (fp16: scale clamps to 0)
    x[1, gs:2 * gs] = 1e-6                       # constant tiny group
    x[2, :gs] = x[2, :gs].abs() + 0.5            # single-signed groups
    x[3, gs:2 * gs] = -(x[3, gs:2 * gs].abs() + 0.5)
    x[4, : gs // 2] = 2.5                        # exact .5 ties after / s
    return x.to(dtype)


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("gs", GROUP_SIZES)
def test_group_size_special_values(gs, dtype, sym, bits):
    check(special((48, 8 * gs), gs, 17 + gs + bits, dtype), gs, sym, bits)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("gs", GROUP_SIZES)
def test_group_size_ragged_batch(gs, dtype):
    """One ragged launch over many tensors (incl. 1-D, odd G) == oracle for every tensor."""
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device(DEV, 0)
    shapes = [(6 * gs,)] * 3 + [(40, 12 * gs), (7, 3 * gs), (300, 2 * gs), (1, gs), (5, 33 * gs), (9, 8 * gs)]
    inputs = {f"t{i}": rand(s, 500 + i, 0.02, dtype).to(dev) for i, s in enumerate(shapes)}
    for bits in (4, 8):
        for sym in (False, True):
            b = PackedBatch(inputs, bits=bits, symmetric=sym, parity=True, group_size=gs)
            b.run()
            torch.cuda.synchronize()
            qmin = -(1 << (bits - 1)) if sym else 0
            for name, res in b.results().items():
                assert int(res["group_size"]) == gs
                ref = orc.quantize(inputs[name].cpu(), bits=bits, group_size=gs, symmetric=sym)
                assert torch.equal(res["tensor_q"].cpu(), ref["tensor_q"]), name
                assert torch.equal(res["zero_points"].cpu(), ref["zero_points"]), name
                assert gio.same_bits(res["scales"].cpu(), ref["scales"]), name
                assert torch.equal(res["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], bits, qmin)), name
                assert torch.equal(res["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], bits, qmin)), name


@pytest.mark.parametrize("gs", GROUP_SIZES)
def test_group_size_model_packed_one_launch(gs):
    """quantize_model_packed routes the whole set through the ragged launch for any
    streaming group size; results equal quantize_packed tensor by tensor."""
    q = Q(bits=4, group_size=gs, symmetric=False)
    tensors = {f"w{i}": rand(s, 900 + i, 0.02) for i, s in enumerate([(64, 4 * gs), (3 * gs,), (9, 5 * gs)])}
    out = q.quantize_model_packed(tensors)
    for n, t in tensors.items():
        one = q.quantize_packed(t)
        for f in ("qweight", "qzeros", "scales"):
            assert torch.equal(out[n][f].cpu(), one[f].cpu()), (n, f)


@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("gs", GROUP_SIZES)
def test_group_size_clip_search_vs_oracle(gs, dtype, sym):
    """Opt-in clip search on the streaming kernel at other group sizes: the canonical
    error tree (8-element chunks, then the pairwise tree over the gs / 8 chunks) matches
    the oracle bit for bit."""
    x = rand((24, 8 * gs), 4242 + gs + sym, 1.0, dtype)
    x[0, :gs] = float("nan")
    x[1, gs:2 * gs] = 0.0
    q = Q(bits=4, group_size=gs, symmetric=sym, scale_method="search")
    ref = orc.quantize(x, bits=4, group_size=gs, symmetric=sym, search=(20, 10))
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])


@pytest.mark.parametrize("gs", GROUP_SIZES)
def test_group_size_full_size_vs_oracle(gs):
    """A full Llama-3-8B MLP shape: single launch == ragged launch bitwise, the whole
    tensor equals the oracle, and the dequantized error stays within the RTN bound."""
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device(DEV, 0)
    g = torch.Generator(device=dev).manual_seed(gs)
    x = (torch.randn(14336, 4096, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    q = Q(bits=4, group_size=gs, symmetric=False)
    pk = q.quantize_packed(x)
    b = PackedBatch({"x": x}, bits=4, symmetric=False, group_size=gs)
    b.run()
    torch.cuda.synchronize()
    for f in ("qweight", "qzeros", "scales"):
        assert torch.equal(b.out["x"][f], pk[f]), f
    ref = orc.quantize(x.cpu(), bits=4, group_size=gs, symmetric=False)
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], 4, 0))
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], 4, 0))
    assert torch.equal(pk["scales"].cpu(), ref["scales"])
    del ref
    dq = q.dequantize_packed(pk)
    s = pk["scales"].float().repeat_interleave(gs, dim=1)
    # same RTN bound as the gs-128 full-size test (tests/test_gpu_parity.py): s/2 plus the
    # bf16 roundings inside the zero point and x/s + z
    assert bool(((dq - x.float()).abs() <= s * 0.7 + 1e-6).all())
