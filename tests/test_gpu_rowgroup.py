"""The row-segment kernel (awq_rowgroup.hip awq_rowgroup_kernel): bf16 / fp16 / fp32 with group
sizes outside {32, 64, 128, 256} (up to 512; fp32 up to 256) and K % 8 != 0 rows — the
shapes that round 1 sent to the one-wave-per-group generic kernel plus int32 staging and
pack passes.  Reference arithmetic: awq.py:173-250 per group, awq.py:286-374 for the row
layout (zero-padded tail group).

Bar: bit-exact vs the oracle for tensor_q / zero_points / fp16 scales (quantize) and for
the packed words (quantize_packed, which must not need staging buffers here), every dtype,
4 / 8 bits, sym / asym, special values; a full-size 14336 x 4096 tensor at group size 100
compared whole.  (The reference's own group-size-100 outputs are pinned separately by the
golden cases in tests/test_gpu_parity.py::test_golden_case.)"""
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
    return AWQQuantizer(device=DEV, logger_level="ERROR", **kw)


def rand(shape, seed, scale=1.0, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


def specials(x, seed):
    x = x.float()
    flat = x.view(-1)
    g = torch.Generator().manual_seed(seed)
    idx = torch.randperm(flat.numel(), generator=g)[: max(6, flat.numel() // 400)]
    kinds = [float("nan"), float("inf"), float("-inf"), 0.0, -0.0, 1e-30]
    for i, j in enumerate(idx.tolist()):
        flat[j] = kinds[i % len(kinds)]
    x[0, : min(40, x.shape[1])] = 0.0           # constant (all-zero) group
    return x


CASES = [  # (dtype, shape, group size) — K % gs != 0 tails, K % 8 != 0, odd and large groups
    (torch.bfloat16, (37, 1000), 100), (torch.bfloat16, (5, 4099), 100), (torch.bfloat16, (9, 777), 3),
    (torch.bfloat16, (64, 1536), 96), (torch.bfloat16, (7, 2000), 500), (torch.bfloat16, (3, 1024), 512),
    (torch.bfloat16, (11, 900), 24), (torch.bfloat16, (13, 4100), 128), (torch.bfloat16, (200, 61), 7),
    (torch.float16, (37, 1000), 100), (torch.float16, (6, 3001), 200), (torch.float16, (17, 250), 50),
    (torch.float32, (37, 1000), 100), (torch.float32, (9, 2050), 256), (torch.float32, (4, 777), 37),
    (torch.bfloat16, (4097,), 100), (torch.bfloat16, (3, 5, 70), 48),
]


def _assert_parity(x, gs, bits, sym):
    from awq_quantizer import _hip
    q = Q(bits=bits, group_size=gs, symmetric=sym)
    ref = orc.quantize(x, bits=bits, group_size=gs, symmetric=sym)
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
    rows = 1 if x.dim() <= 1 else x.shape[0]
    assert _hip.packs_directly(x.dtype, rows, x.numel() // rows, gs)
    pk = q.quantize_packed(x)
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"].reshape(rows, -1), bits, q.qmin))
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], bits, q.qmin))
    assert gio.same_bits(pk["scales"].cpu(), ref["scales"])


@pytest.mark.parametrize("bits,sym", [(4, False), (4, True), (8, False), (8, True)], ids=str)
@pytest.mark.parametrize("dtype,shape,gs", CASES, ids=str)
def test_rowgroup_vs_oracle(dtype, shape, gs, bits, sym):
    _assert_parity(rand(shape, hash((shape, gs, bits, sym)) & 0xFFFF, 0.5, dtype), gs, bits, sym)


@pytest.mark.parametrize("bits,sym", [(4, False), (4, True), (8, True)], ids=str)
@pytest.mark.parametrize("dtype,gs", [(torch.bfloat16, 100), (torch.float16, 100), (torch.float32, 60),
                                      (torch.bfloat16, 300)], ids=str)
def test_rowgroup_special_values(dtype, gs, bits, sym):
    x = specials(rand((24, 1300), 5 + gs, 1.0), 9 + bits).to(dtype)
    _assert_parity(x, gs, bits, sym)


def test_rowgroup_full_size_gs100():
    """14336 x 4096 (a Llama-3-8B MLP weight) at group size 100: 41 groups per row, the
    last padded (K % 100 = 96); the whole tensor equals the oracle."""
    dev = torch.device(DEV, 0)
    g = torch.Generator(device=dev).manual_seed(100)
    x = (torch.randn(14336, 4096, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    q = Q(bits=4, group_size=100, symmetric=False)
    pk = q.quantize_packed(x)
    ref = orc.quantize(x.cpu(), bits=4, group_size=100, symmetric=False)
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], 4, 0))
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], 4, 0))
    assert torch.equal(pk["scales"].cpu(), ref["scales"])


def test_generic_kernel_still_serves_the_rest():
    """fp64, groups larger than the row-segment stage, and tuning no_rowgroup=1 take the generic
    kernel (packed outputs written directly per span of groups, no staging) with the same results."""
    from awq_quantizer import _hip
    assert _hip.packs_directly(torch.float64, 4, 1000, 100)
    assert _hip.packs_directly(torch.bfloat16, 4, 5000, 1000)
    assert _hip.packs_directly(torch.float32, 4, 1000, 500)
    _assert_parity_generic = lambda x, gs: orc.quantize(x, bits=4, group_size=gs, symmetric=False)
    for x, gs in ((rand((4, 1000), 1, 1.0, torch.float64), 100), (rand((4, 5000), 2), 1000)):
        q = Q(bits=4, group_size=gs, symmetric=False)
        ref = _assert_parity_generic(x, gs)
        assert torch.equal(q.quantize(x)["tensor_q"], ref["tensor_q"])
        pk = q.quantize_packed(x)
        assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], 4, 0))
    with _hip.tuning(no_rowgroup=1):
        x = rand((37, 1000), 3)
        ref = orc.quantize(x, bits=4, group_size=100, symmetric=False)
        assert torch.equal(Q(bits=4, group_size=100, symmetric=False).quantize(x)["tensor_q"], ref["tensor_q"])


@pytest.mark.parametrize("gpt", [24, 40, 64], ids=str)
@pytest.mark.parametrize("dtype,shape,gs", [(torch.bfloat16, (37, 1000), 100), (torch.bfloat16, (9, 4100), 96),
                                            (torch.float16, (5, 3001), 60), (torch.float32, (6, 2050), 48),
                                            (torch.bfloat16, (200, 61), 7)], ids=str)
def test_rowgroup_groups_per_tile_override(dtype, shape, gs, gpt):
    """Groups per tile that are not powers of two (rg_gpt tuning override, any multiple
    of 8): P = the largest power of two <= 64 / the tile's groups, the row's light last
    tile with more lanes per group, word-aligned tile boundaries — same bits as the oracle."""
    from awq_quantizer import _hip
    with _hip.tuning(rg_gpt=gpt):
        for bits, sym in ((4, False), (8, True)):
            _assert_parity(rand(shape, gpt + gs + bits, 0.5, dtype), gs, bits, sym)


@pytest.mark.parametrize("dtype,shape,gs", CASES, ids=str)
def test_rowgroup_pass1_split_runs(dtype, shape, gs):
    """Pass 1 with the tile's lanes split evenly over its groups (tuning rg_p1=2: NT / groups
    lanes per group, LDS ds_max / ds_min merges, parameters by one lane per group) against
    the same oracle as the default by-groups pass 1."""
    from awq_quantizer import _hip
    with _hip.tuning(rg_p1=2):
        for bits, sym in ((4, False), (8, True)):
            _assert_parity(rand(shape, gs + bits + 7, 0.5, dtype), gs, bits, sym)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=str)
@pytest.mark.parametrize("K,gs", [(4096, 100), (4096, 96), (4096, 48), (4096, 200), (3000, 100), (4104, 100),
                                  (4098, 100), (2562, 52)], ids=str)
def test_rowgroup_whole_row_tiles(dtype, K, gs):
    """Whole-row two-wave tiles (K >= 2 560, <= 64 groups): the exactly-4-chunks-per-lane
    stage (K = 4096: 512 chunks on 128 lanes), the uniform full sweeps of pass 2 and the
    guarded remainder (K = 3000, 4104), the packed-only and parity kernels, special values."""
    x = rand((96, K), K + gs, 0.5, dtype)
    for bits, sym in ((4, False), (8, True)):
        _assert_parity(x, gs, bits, sym)
    _assert_parity(specials(rand((24, K), gs, 1.0), 3).to(dtype), gs, 4, False)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=str)
@pytest.mark.parametrize("K,gs", [(14336, 100), (14336, 60), (8192, 100), (12000, 124), (9001, 58), (14336, 76),
                                  (8192, 60)],
                         ids=str)
def test_rowgroup_long_row_two_wave_tiles(dtype, K, gs):
    """Rows longer than 64 groups with L % 8 != 0 (56 <= L <= 128) take two-wave tiles of
    <= 9.6 KB (round 4): full tiles, the row's lighter last tile, K % gs != 0 and K % 8 != 0
    tails, 4 / 8 bits, special values — same bits as the oracle."""
    x = rand((24, K), K + gs, 0.5, dtype)
    for bits, sym in ((4, False), (8, True)):
        _assert_parity(x, gs, bits, sym)
    _assert_parity(specials(rand((8, K), gs + 1, 1.0), 5).to(dtype), gs, 4, False)


@pytest.mark.parametrize("tun", [{"rg_ldsdma": 1}, {"rg_ldsdma": 1, "rg_p2reg": 1}, {"rg_p1u": 1}],
                         ids=lambda t: "_".join(t))
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32], ids=str)
@pytest.mark.parametrize("K,gs", [(4096, 100), (4096, 48), (4096, 200), (3000, 100), (14336, 100), (1000, 60),
                                  (203, 50), (4098, 100), (8192, 60)], ids=str)
def test_rowgroup_stage_variants_same_bits(dtype, K, gs, tun):
    """The LDS-DMA stage (the default) gives the bits of the round-3 register stage
    (diagnostics build, rg_ldsdma = 1), whose 4-chunk case feeds pass 2 from registers or
    (rg_p2reg = 1) from LDS; the uniform pass 1 (default where it applies: zero-staged
    padding, also past a segment ending inside a 16-B chunk, K = 4098) the bits of the
    per-lane bounds form (rg_p1u = 1); whole-row, one-wave and partial tiles, the tensor's
    last bytes (K = 203), special values."""
    if dtype == torch.float32 and gs > 256:
        pytest.skip("fp32 row segments take group sizes <= 256")
    from awq_quantizer import _hip
    x = specials(rand((40, K), K + gs + 7, 0.5), 9).to(dtype)
    for bits, sym in ((4, False), (8, True)):
        q = Q(bits=bits, group_size=gs, symmetric=sym)
        a = q.quantize_packed(x)
        with _hip.tuning(**tun):
            b = Q(bits=bits, group_size=gs, symmetric=sym).quantize_packed(x)
        for key in ("qweight", "qzeros"):
            assert torch.equal(a[key], b[key]), key
        assert gio.same_bits(a["scales"], b["scales"])
