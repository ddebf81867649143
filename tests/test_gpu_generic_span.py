"""The generic kernel after its span rewrite (awq_generic.hip awq_generic_kernel): one wave per
span of 32 / bits groups of a row (the groups sharing one qzeros word), qweight / qzeros
packed in the kernel with cross-lane shuffles — no int32 staging, no pack pass.  It serves
fp64 inputs and groups larger than the row-segment stage (> 512; fp32 > 256), and every
dtype under AWQ_NO_ROWGROUP=1.  Reference arithmetic: awq.py:173-250 per group, awq.py:286-374
for the row layout (zero-padded tail group), awq.py:130-171 for numel < group_size.

Bar: bit-exact vs the oracle for tensor_q / zero_points / fp16 scales (quantize) and for the
packed words (quantize_packed without staging buffers): group sizes below 64 lanes, not a
multiple of the pack width, larger than a wave's stride, a row's last span with fewer
groups, 4 / 8 bits, sym / asym, NaN / inf / constant groups, and the clip search."""
import os

import pytest
import torch

import golden_io as gio
from oracle import awq_oracle as orc
from test_gpu_rowgroup import Q, _assert_parity, _need_gpu, rand, specials  # noqa: F401

pytestmark = pytest.mark.gpu

F64_CASES = [  # (shape, group size): spans of 8 (4-bit) / 4 (8-bit) groups, ragged last spans
    ((37, 1000), 100), ((5, 3001), 60), ((9, 4100), 96), ((3, 200), 7), ((4, 1024), 128),
    ((6, 777), 37), ((2, 5000), 1000), ((3, 2048), 32), ((4097,), 100), ((3, 5, 70), 48),
    # group sizes 64 / 128 take the register-resident span (padded tails, K % 8 != 0, G < 8)
    ((5, 1000), 128), ((7, 1001), 64), ((3, 640), 128), ((9, 4096), 64), ((2, 100), 64),
]


@pytest.mark.parametrize("bits,sym", [(4, False), (4, True), (8, False), (8, True)], ids=str)
@pytest.mark.parametrize("shape,gs", F64_CASES, ids=str)
def test_generic_f64_vs_oracle(shape, gs, bits, sym):
    _assert_parity(rand(shape, hash((shape, gs, bits, sym)) & 0xFFFF, 0.5, torch.float64), gs, bits, sym)


@pytest.mark.parametrize("bits,sym", [(4, False), (8, True)], ids=str)
@pytest.mark.parametrize("gs", [100, 13, 640, 128, 64], ids=str)
def test_generic_f64_special_values(gs, bits, sym):
    x = specials(rand((24, 1300), 7 + gs, 1.0), 11 + bits).to(torch.float64)
    _assert_parity(x, gs, bits, sym)


@pytest.mark.parametrize("dtype,shape,gs", [(torch.bfloat16, (7, 5000), 1000), (torch.float16, (3, 4500), 900),
                                            (torch.float32, (5, 3000), 300), (torch.bfloat16, (2, 9000), 4500)],
                         ids=str)
def test_generic_large_groups(dtype, shape, gs):
    """Groups beyond the row-segment stage: lanes stride over a group several times."""
    for bits, sym in ((4, False), (8, True)):
        _assert_parity(rand(shape, gs + bits, 0.5, dtype), gs, bits, sym)


@pytest.mark.parametrize("dtype,shape,gs", [(torch.bfloat16, (37, 1000), 100), (torch.float16, (9, 777), 3),
                                            (torch.float32, (13, 4100), 128)], ids=str)
def test_generic_forced_by_tuning(dtype, shape, gs):
    """tuning no_rowgroup=1 sends the row-segment shapes to the generic kernel: same bits."""
    from awq_quantizer import _hip
    with _hip.tuning(no_rowgroup=1):
        for bits, sym in ((4, False), (4, True), (8, False)):
            _assert_parity(specials(rand(shape, gs + bits, 0.5), 3).to(dtype), gs, bits, sym)


@pytest.mark.parametrize("gs", [100, 64], ids=str)
def test_generic_f64_search_packed(gs):
    """Clip search on fp64 (generic kernel): the packed words are the oracle's search result packed."""
    from awq_quantizer import _hip
    x = rand((9, 1000), 21 + gs, 0.5, torch.float64)
    rows, K = x.shape
    G = -(-K // gs)
    ref = orc.quantize(x, bits=4, group_size=gs, symmetric=False, search=(20, 10))
    d = x.to("cuda")
    qw = torch.empty(rows, -(-K // 8), dtype=torch.int32, device="cuda")
    qz = torch.empty(rows, -(-G // 8), dtype=torch.int32, device="cuda")
    sc = torch.empty(rows, G, dtype=torch.float16, device="cuda")
    _hip.quantize_search(d, rows, K, gs, 4, False, 20, 10, qweight=qw, qzeros=qz, scales=sc)
    torch.cuda.synchronize()
    assert torch.equal(qw.cpu(), orc.pack_rows(ref["tensor_q"].reshape(rows, -1), 4, 0))
    assert torch.equal(qz.cpu(), orc.pack_rows(ref["zero_points"], 4, 0))


@pytest.mark.parametrize("bits,sym", [(4, False), (4, True), (8, False), (8, True)], ids=str)
@pytest.mark.parametrize("dtype,shape,gs", [(torch.bfloat16, (64, 4096), 128), (torch.float16, (33, 1024), 32),
                                            (torch.bfloat16, (17, 2000), 200), (torch.float32, (5, 4096), 256),
                                            (torch.bfloat16, (9, 1000), 100), (torch.bfloat16, (7, 1001), 91),
                                            (torch.float64, (6, 1024), 64), (torch.bfloat16, (13, 2000), 50),
                                            (torch.float16, (11, 1008), 7), (torch.bfloat16, (4, 4096), 100),
                                            (torch.bfloat16, (6, 64), 3), (torch.float32, (8, 4104), 57),
                                            (torch.bfloat16, (3, 512), 4)], ids=str)
def test_dequantize_packed_vs_oracle(dtype, shape, gs, bits, sym):
    """dequantize_packed (awq.py:459-539 arithmetic): rows of whole qweight words (K a multiple
    of 32 / bits) take the batched quad kernel — word-aligned groups, quad-aligned groups
    (L % 4 == 0) or any L >= 4 (a quad meeting two groups) — the rest (L < 4, ragged K) the
    per-element kernel; NaN / inf /
    constant groups included.  Bit-exact (NaN payloads compared as NaN) vs the oracle's
    dequantize of the oracle's quantize, its int32 values taken through the packed format
    first (a nibble / byte holds (v - qmin) mod 2^bits: the INT_MIN of an inf / inf element
    becomes qmin, so such an element of an inf-scale group dequantizes to NaN, not -inf)."""
    x = specials(rand(shape, gs + bits + sym, 0.5), 5).to(dtype)
    q = Q(bits=bits, group_size=gs, symmetric=sym)
    ref = dict(orc.quantize(x, bits=bits, group_size=gs, symmetric=sym))
    for key in ("tensor_q", "zero_points"):
        ref[key] = (((ref[key].long() - q.qmin) & ((1 << bits) - 1)) + q.qmin).to(torch.int32)
    dq = q.dequantize_packed(q.quantize_packed(x)).cpu()
    assert gio.same_bits(dq, orc.dequantize(ref))


@pytest.mark.parametrize("other", [1, 2], ids=["strided", "register"])
@pytest.mark.parametrize("gs", [64, 128], ids=str)
def test_generic_f64_reg_span_matches_strided(gs, other):
    """At group sizes 64 / 128 the default fp64 LDS span, the strided span kernel (tuning
    gen_noreg=1) and the register-resident span (gen_noreg=2) give the same bits on a ragged
    shape with special values."""
    from awq_quantizer import _hip
    x = specials(rand((33, 1000), gs, 1.0), 17).to(torch.float64)
    q = Q(bits=4, group_size=gs, symmetric=False)
    a = q.quantize_packed(x)
    with _hip.tuning(gen_noreg=other):
        b = Q(bits=4, group_size=gs, symmetric=False).quantize_packed(x)
    for key in ("qweight", "qzeros"):
        assert torch.equal(a[key], b[key])
    assert gio.same_bits(a["scales"], b["scales"])


@pytest.mark.parametrize("variant", range(1, 10), ids=lambda v: f"dq{v}")
@pytest.mark.parametrize("bits", [4, 8], ids=str)
def test_dequantize_packed_kernel_variants(variant, bits):
    """Every word-aligned dequantize kernel (tuning dq_words_v1 1..9: round-2 words, LDS-staged,
    four-output lanes, batched lanes, with / without XCD block orders) gives the oracle's bits,
    on a shape whose last block is partial (rows * K / 4 quads not a multiple of any block)
    with special values."""
    from awq_quantizer import _hip
    x = specials(rand((37, 1536), variant + bits, 0.5), 11).to(torch.bfloat16)
    q = Q(bits=bits, group_size=128, symmetric=False)
    pk = q.quantize_packed(x)
    ref = dict(orc.quantize(x, bits=bits, group_size=128, symmetric=False))
    for key in ("tensor_q", "zero_points"):
        ref[key] = (((ref[key].long() - q.qmin) & ((1 << bits) - 1)) + q.qmin).to(torch.int32)
    with _hip.tuning(dq_words_v1=variant):
        dq = q.dequantize_packed(pk).cpu()
    assert gio.same_bits(dq, orc.dequantize(ref))


@pytest.mark.parametrize("bits", [4, 8], ids=str)
@pytest.mark.parametrize("shape,gs", [((33, 1000), 100), ((9, 777), 7), ((5, 1001), 2), ((6, 2049), 256),
                                      ((4, 1600), 200), ((7, 3000), 500), ((3, 95), 96)], ids=str)
def test_f64_lds_span_vs_oracle_and_strided(shape, gs, bits):
    """fp64 at group sizes other than 64 / 128 (the LDS span kernel: 4-bit L <= 256, 8-bit
    L <= 512) against the oracle (tensor_q, zero points, scales, packed words) and against
    the strided span (tuning gen_noreg=1), ragged K and special values included."""
    from awq_quantizer import _hip
    x = specials(rand(shape, gs + bits, 1.0), 23 + gs).to(torch.float64)
    for sym in (False, True):
        _assert_parity(x, gs, bits, sym)
        a = Q(bits=bits, group_size=gs, symmetric=sym).quantize_packed(x)
        with _hip.tuning(gen_noreg=1):
            b = Q(bits=bits, group_size=gs, symmetric=sym).quantize_packed(x)
        for key in ("qweight", "qzeros"):
            assert torch.equal(a[key], b[key])
        assert gio.same_bits(a["scales"], b["scales"])
