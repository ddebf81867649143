"""fp32 weights on the streaming kernel (group sizes 32/64/128/256, K % group_size == 0):
bit-exact against the oracle.

fp32 is the reference's arithmetic without any narrowing (torch fp32 ops, awq.py:173-250):
x / s is the IEEE division, t + z one fp32 add.  Two places where the 16-bit formats'
shortcuts would be wrong for fp32 are pinned here: the symmetric field rint(t) + 8 (t + 8
is not exact for a 24-bit t: 0.5 + 2^-24 + 8 rounds to 8.5), and constant groups whose
scale clamps to 1e-10 (x / s overflows to +-inf and must clamp, not turn into NaN).  The
golden fixtures' fp32 cases (tests/test_gpu_parity.py::test_golden_case) also run here now.
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


def rand32(shape, seed, scale=0.02):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


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


def test_f32_takes_the_streaming_kernel():
    from awq_quantizer import _hip
    for gs in (32, 64, 128, 256):
        assert _hip.ragged_eligible(torch.float32, 1024, 16 * gs, gs)
    assert _hip.ragged_eligible(torch.float32, 1024, 4000, 128)       # padded rows (K % 8 == 0)
    assert not _hip.ragged_eligible(torch.float32, 1024, 4001, 128)   # K % 8 != 0: generic


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("gs", [32, 64, 128, 256])
def test_f32_vs_oracle(gs, sym, bits):
    shapes = [(64, 32 * gs), (7, 3 * gs), (11, gs), (3, 9 * gs), (33, 8 * gs), (6 * gs,), (2, 3, 2 * gs),
              (129, 2 * gs)]
    for i, shape in enumerate(shapes):
        check(rand32(shape, 7000 + 31 * gs + 10 * i + 2 * sym + bits), gs, sym, bits)


def special32(shape, gs, seed):
    x = rand32(shape, seed, 1.0)
    flat = x.view(-1)
    g = torch.Generator().manual_seed(seed + 1)
    idx = torch.randperm(flat.numel(), generator=g)[: max(8, flat.numel() // 300)]
    kinds = [float("nan"), float("inf"), float("-inf"), 3e38, -3e38, 1e-40, 0.0, -0.0]
    for i, j in enumerate(idx.tolist()):
        flat[j] = kinds[i % len(kinds)]
    x[0, :gs] = 0.0                                 # all-zero group: s = 1e-10
    x[1, gs:2 * gs] = 5e30                          # constant huge group: x / 1e-10 overflows
    x[2, :gs] = -7e29
    x[3, gs:2 * gs] = 1e-6                          # constant tiny group
    x[4, :gs] = x[4, :gs].abs() + 0.5               # single-signed groups
    x[5, gs:2 * gs] = -(x[5, gs:2 * gs].abs() + 0.5)
    return x


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("gs", [32, 128, 256])
def test_f32_special_values(gs, sym, bits):
    check(special32((48, 8 * gs), gs, 31 + gs + bits), gs, sym, bits)


@pytest.mark.parametrize("bits", [4, 8])
def test_f32_symmetric_near_ties(bits):
    """sym: groups with max |x| = qmax + 0.5 (s = 1 exactly) holding values a few ulps
    above / below k + 0.5: rint(t) + 2^(bits-1) is right, rint(t + 2^(bits-1)) is not
    (9 / 144 elements differ at 4 / 8 bits; checked against the oracle on the CPU)."""
    gs = 128
    qmax = (1 << (bits - 1)) - 1
    a = qmax + 0.5                                   # s = 2a / (2^bits - 1) = 1 exactly
    rows = []
    for k in range(-3, 3):
        base = torch.full((gs,), float(k) + 0.5)
        nud = torch.arange(gs, dtype=torch.float32) - gs // 2
        v = torch.nextafter(base, torch.full_like(base, 1e9 if k % 2 else -1e9))
        v = v + nud * 2.0 ** -22
        v[0], v[1] = a, -a
        rows.append(v)
    x = torch.stack(rows)
    check(x, gs, True, bits)
    check(x, gs, False, bits)


def test_f32_ragged_and_mixed_dtypes():
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device(DEV, 0)
    shapes = [(768,)] * 3 + [(768, 768), (300, 256), (7, 384), (9, 1792), (1, 128)]
    inputs = {f"t{i}": rand32(s, 600 + i).to(dev) for i, s in enumerate(shapes)}
    for bits in (4, 8):
        for sym in (False, True):
            b = PackedBatch(inputs, bits=bits, symmetric=sym, parity=True)
            b.run()
            torch.cuda.synchronize()
            qmin = -(1 << (bits - 1)) if sym else 0
            for name, res in b.results().items():
                ref = orc.quantize(inputs[name].cpu(), bits=bits, group_size=128, symmetric=sym)
                assert torch.equal(res["tensor_q"].cpu(), ref["tensor_q"]), name
                assert torch.equal(res["zero_points"].cpu(), ref["zero_points"]), name
                assert gio.same_bits(res["scales"].cpu(), ref["scales"]), name
                assert torch.equal(res["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], bits, qmin)), name
                assert torch.equal(res["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], bits, qmin)), name
    mixed = {"a": rand32((256, 512), 1), "b": rand32((512,), 2).to(torch.bfloat16),
             "c": rand32((64, 256), 3).to(torch.float16), "d": rand32((5, 300), 4)}
    out = Q(bits=4, symmetric=False).quantize_model_packed(mixed)
    for name, t in mixed.items():
        ref = orc.quantize(t, bits=4, group_size=128, symmetric=False)
        rows = 1 if t.dim() == 1 else t.shape[0]
        assert torch.equal(out[name]["qweight"].cpu(), orc.pack_rows(ref["tensor_q"].reshape(rows, -1), 4, 0)), name


@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("gs", [64, 128])
def test_f32_clip_search_vs_oracle(gs, sym):
    x = rand32((24, 8 * gs), 4343 + gs + sym, 1.0)
    x[0, :gs] = float("nan")
    x[1, gs:2 * gs] = 0.0
    q = Q(bits=4, group_size=gs, symmetric=sym, scale_method="search")
    ref = orc.quantize(x, bits=4, group_size=gs, symmetric=sym, search=(20, 10))
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])


def test_f32_full_size_row_sample():
    """A full 14336 x 4096 fp32 tensor (235 MB): single == ragged launch bitwise, a row
    sample equals the oracle."""
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device(DEV, 0)
    g = torch.Generator(device=dev).manual_seed(32)
    x = torch.randn(14336, 4096, generator=g, device=dev) * 0.02
    q = Q(bits=4, symmetric=False)
    pk = q.quantize_packed(x)
    b = PackedBatch({"x": x}, bits=4, symmetric=False)
    b.run()
    torch.cuda.synchronize()
    for f in ("qweight", "qzeros", "scales"):
        assert torch.equal(b.out["x"][f], pk[f]), f
    rows = torch.arange(0, 14336, 1499)
    ref = orc.quantize(x[rows].cpu(), bits=4, group_size=128, symmetric=False)
    assert torch.equal(pk["qweight"][rows].cpu(), orc.pack_rows(ref["tensor_q"], 4, 0))
    assert torch.equal(pk["qzeros"][rows].cpu(), orc.pack_rows(ref["zero_points"], 4, 0))
    assert torch.equal(pk["scales"][rows].cpu(), ref["scales"])
