"""Parity of the HIP path (libawq_hip.so via the drop-in AWQQuantizer) with the oracle
and the reference's golden outputs.  Needs a gfx950 GPU: `pytest -m gpu`.

Bar: bit-exact int32 tensor_q / zero_points, fp16 scales (NaN bits included), fp32
dequantize; packed qweight/qzeros equal the oracle's packing of the oracle's values.
"""
import os

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
    _hip.require_device(torch.device("cuda", 0))   # raises unless gfx950 + library present


def Q(**kw):
    from awq_quantizer.quantization import AWQQuantizer
    kw.setdefault("device", DEV)
    return AWQQuantizer(logger_level="ERROR", **kw)


def rand_bf16(shape, seed, scale=1.0, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


# ---------------------------------------------------------------- golden fixtures
@pytest.mark.parametrize("case", gio.ok_cases(), ids=lambda c: c["name"])
def test_golden_case(case):
    x = gio.case_input(case)
    p = dict(case["params"])
    res = Q(**p).quantize(x)
    T = gio.tensors()
    name = case["name"]
    assert torch.equal(res["tensor_q"], T[name + ".tensor_q"])
    assert torch.equal(res["zero_points"], T[name + ".zero_points"])
    assert gio.same_bits(res["scales"], T[name + ".scales"])
    assert res["tensor_q"].dtype == torch.int32 and res["scales"].dtype == torch.float16
    if name + ".dq" in T:
        dq = Q(**p).dequantize(res)
        assert gio.same_bits(dq, T[name + ".dq"])
    elif case.get("dequantize") == "IndexError":
        with pytest.raises(IndexError):
            Q(**p).dequantize(res)


@pytest.mark.parametrize("rec", gio.manifest()["hashed"], ids=lambda r: r["name"])
def test_golden_hashed(rec):
    x = gio.hashed_input(rec)
    assert gio.sha(x) == rec["sha_x"]
    q = Q(**rec["params"])
    res = q.quantize(x)
    assert gio.sha(res["tensor_q"]) == rec["sha_tensor_q"]
    assert gio.sha(res["scales"]) == rec["sha_scales"]
    assert gio.sha(res["zero_points"]) == rec["sha_zero_points"]
    assert gio.sha(q.dequantize(res)) == rec["sha_dq"]


def test_percentile_mode_raises_like_reference():
    with pytest.raises(TypeError):
        Q(zero_point="percentile").quantize(rand_bf16((4, 256), 0))
    assert Q(zero_point="percentile").quantize_model({"a": rand_bf16((4, 256), 0)}) == {}


def test_quantize_model_skip_semantics():
    m = {"w": rand_bf16((8, 256), 30), "i": torch.arange(256, dtype=torch.int32),
         "s": rand_bf16((10, 10), 31), "e": torch.zeros(0, dtype=torch.bfloat16), "b": rand_bf16((256,), 32)}
    out = Q(symmetric=False).quantize_model(m)
    assert sorted(out) == gio.manifest()["quantize_model"]["asym"]


# ---------------------------------------------------------------- oracle, random shapes
FAST_SHAPES = [(1024, 4096), (4096, 768), (768,), (3072,), (7, 1792), (3, 1280), (5, 384), (9, 128),
               (33, 11 * 128), (2, 8, 256), (64, 14336), (1, 65536), (13, 1280), (6, 2560), (40, 256),
               (7, 640), (5, 1152), (77, 768), (3, 896)]


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("shape", FAST_SHAPES, ids=str)
def test_fast_path_vs_oracle(shape, sym, bits):
    x = rand_bf16(shape, hash((shape, sym, bits)) & 0xFFFF, 0.02)
    ref = orc.quantize(x, bits=bits, group_size=128, symmetric=sym)
    q = Q(bits=bits, symmetric=sym)
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
    pk = q.quantize_packed(x)
    qmin = q.qmin
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], bits, qmin))
    zz = ref["zero_points"]
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(zz, bits, qmin))
    assert gio.same_bits(pk["scales"].cpu(), ref["scales"])
    dq_packed = q.dequantize_packed(pk).cpu()
    assert gio.same_bits(dq_packed, orc.dequantize(ref))


def special_tensor(shape, seed):
    """bf16 with NaN, +-inf, huge, subnormal and constant groups sprinkled in."""
    x = rand_bf16(shape, seed, 1.0).float()
    flat = x.view(-1)
    g = torch.Generator().manual_seed(seed + 1)
    n = flat.numel()
    idx = torch.randperm(n, generator=g)[: max(8, n // 500)]
    kinds = [float("nan"), float("inf"), float("-inf"), 3e38, -3e38, 1e-39, 0.0, -0.0]
    for i, j in enumerate(idx.tolist()):
        flat[j] = kinds[i % len(kinds)]
    x[0, :128] = 0.0                        # all-zero group
    x[min(1, shape[0] - 1), 128:256] = 1e-6  # constant tiny group
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [False, True])
def test_fast_path_special_values(sym, bits):
    x = special_tensor((64, 1024), 7 + bits + sym)
    ref = orc.quantize(x, bits=bits, group_size=128, symmetric=sym)
    q = Q(bits=bits, symmetric=sym)
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
    pk = q.quantize_packed(x)
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], bits, q.qmin))
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], bits, q.qmin))


GENERIC = [(torch.float16, (33, 300), 128), (torch.float32, (17, 1000), 64), (torch.float64, (5, 777), 100),
           (torch.bfloat16, (12, 4000), 256), (torch.bfloat16, (12, 300), 128), (torch.float16, (256, 4096), 128),
           (torch.bfloat16, (3, 2, 50), 32), (torch.float32, (1, 5000), 1000)]


@pytest.mark.parametrize("dtype,shape,gs", GENERIC, ids=str)
@pytest.mark.parametrize("sym", [False, True])
def test_generic_path_vs_oracle(dtype, shape, gs, sym):
    x = rand_bf16(shape, 99, 0.5, dtype)
    ref = orc.quantize(x, bits=4, group_size=gs, symmetric=sym)
    q = Q(bits=4, group_size=gs, symmetric=sym)
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
    pk = q.quantize_packed(x)
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], 4, q.qmin))
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], 4, q.qmin))


# ---------------------------------------------------------------- ragged launch
def test_ragged_batch_matches_single_and_oracle():
    from awq_quantizer.quantization.batch import PackedBatch
    shapes = [(768,)] * 5 + [(768, 768), (3072, 768), (768, 3072), (2050, 768), (3072,), (128,), (9, 1792),
                             (4, 128), (1, 640)]
    dev = torch.device(DEV, 0)
    inputs = {f"t{i}": rand_bf16(s, 200 + i, 0.02).to(dev) for i, s in enumerate(shapes)}
    for bits in (4, 8):
        for sym in (False, True):
            b = PackedBatch(inputs, bits=bits, symmetric=sym, parity=True)
            b.run()
            torch.cuda.synchronize()
            q = Q(bits=bits, symmetric=sym)
            for name, res in b.results().items():
                x = inputs[name].cpu()
                ref = orc.quantize(x, bits=bits, group_size=128, symmetric=sym)
                assert torch.equal(res["tensor_q"].cpu(), ref["tensor_q"]), name
                assert torch.equal(res["zero_points"].cpu(), ref["zero_points"]), name
                assert gio.same_bits(res["scales"].cpu(), ref["scales"]), name
                assert torch.equal(res["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], bits, q.qmin)), name
                assert torch.equal(res["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], bits, q.qmin)), name


def test_ragged_rerun_idempotent():
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device(DEV, 0)
    inputs = {f"t{i}": rand_bf16(s, 300 + i).to(dev) for i, s in enumerate([(1024, 4096), (4096,), (50, 768)])}
    b = PackedBatch(inputs, bits=4, symmetric=False)
    b.run()
    first = {k: {kk: vv.clone() for kk, vv in v.items()} for k, v in b.out.items()}
    for _ in range(3):
        b.run()
    torch.cuda.synchronize()
    for k, v in b.out.items():
        for kk, vv in v.items():
            assert torch.equal(vv, first[k][kk])


# ---------------------------------------------------------------- full-size properties
@pytest.mark.parametrize("shape", [(14336, 4096), (4096, 14336), (128256, 4096)], ids=str)
def test_full_size_properties(shape):
    """BASELINE-size tensors (Llama-3-8B MLP / embedding): single launch == ragged launch
    bitwise; dequantized error <= s/2 per element (RTN bound) except clamped extremes;
    the whole tensor matches the oracle bit for bit."""
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device(DEV, 0)
    g = torch.Generator(device=dev).manual_seed(5)
    x = (torch.randn(*shape, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    q = Q(bits=4, symmetric=False)
    pk = q.quantize_packed(x)
    b = PackedBatch({"x": x}, bits=4, symmetric=False)
    b.run()
    torch.cuda.synchronize()
    assert torch.equal(b.out["x"]["qweight"], pk["qweight"])
    assert torch.equal(b.out["x"]["qzeros"], pk["qzeros"])
    assert torch.equal(b.out["x"]["scales"], pk["scales"])
    dq = q.dequantize_packed(pk)
    s = pk["scales"].float().repeat_interleave(128, dim=1)
    err = (dq - x.float()).abs()
    # RTN bound of the reference arithmetic: s/2, plus the bf16 rounding of mn/s inside the
    # zero point (z can land 0.53 away from -mn/s) and of x/s + z; measured max 0.616 s
    assert bool((err <= s * 0.7 + 1e-6).all())
    del dq, s, err
    ref = orc.quantize(x.cpu(), bits=4, group_size=128, symmetric=False)
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], 4, 0))
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], 4, 0))
    assert torch.equal(pk["scales"].cpu(), ref["scales"])


@pytest.mark.parametrize("blocks,gs,dtype", [("1", 128, torch.bfloat16), ("3", 128, torch.bfloat16),
                                             ("8", 128, torch.bfloat16), ("3", 32, torch.bfloat16),
                                             ("5", 256, torch.float16), ("3", 64, torch.float32)], ids=str)
def test_grid_stride_loop(blocks, gs, dtype):
    """Force a tiny grid (tuning max_blocks) so every wave walks many tiles/tensors."""
    from awq_quantizer import _hip
    with _hip.tuning(max_blocks=int(blocks)):
        _grid_stride_case(gs, dtype)


def _grid_stride_case(gs, dtype):
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device(DEV, 0)
    shapes = [s for s in [(300, 4096), (768,), (50, 768), (7, 1792), (4096,), (33, 384)] if s[-1] % gs == 0]
    inputs = {f"t{i}": rand_bf16(s, 400 + i, 0.02, dtype).to(dev) for i, s in enumerate(shapes)}
    b = PackedBatch(inputs, bits=4, symmetric=False, parity=True, group_size=gs)
    b.run()
    torch.cuda.synchronize()
    q = Q(bits=4, symmetric=False, group_size=gs)
    for name, x in inputs.items():
        ref = orc.quantize(x.cpu(), bits=4, group_size=gs, symmetric=False)
        o = b.out[name]
        assert torch.equal(o["tensor_q"].cpu(), ref["tensor_q"]), name
        assert torch.equal(o["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], 4, 0)), name
        assert torch.equal(o["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], 4, 0)), name
        assert torch.equal(o["scales"].cpu(), ref["scales"]), name
        pk = q.quantize_packed(x)        # single-tensor launch, same tiny grid
        assert torch.equal(pk["qweight"], o["qweight"]), name


def test_selftest_fast_reciprocal_exhaustive():
    """recip_bf16 (v_rcp + Newton) == IEEE 1/s for every bf16 scale value."""
    from awq_quantizer import _hip
    assert _hip.selftest(0, torch.device(DEV, 0)) == 0


def test_selftest_fast_reciprocal_f16_exhaustive():
    """Round 6: recip_f16 (v_rcp + Newton) == IEEE 1/s for every positive finite fp16 scale (the
    fp16 group parameters' reciprocal, AWQ_F16_PARAMS_FAST)."""
    from awq_quantizer import _hip
    assert _hip.selftest(2, torch.device(DEV, 0)) == 0


def test_stream_copy_helper_copies_exactly():
    """bench.py's copy-ceiling kernel (awq_stream_copy) is a faithful copy, tail included."""
    from awq_quantizer import _hip
    dev = torch.device(DEV, 0)
    for n in (16, 4096, 4096 * 8 * 3 + 48):
        src = torch.randint(-2 ** 31, 2 ** 31 - 1, (n // 4,), dtype=torch.int32, device=dev)
        dst = torch.zeros_like(src)
        _hip.stream_copy(src, dst, torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(src, dst)


def test_stream_ceiling_helper_reads_all_writes_quarter():
    """bench.py's read-dominant ceiling kernel: every 4 KiB of src is read (its four 1-KiB
    quarters xor-folded per lane) and 1 KiB of dst written per 4 KiB."""
    from awq_quantizer import _hip
    dev = torch.device(DEV, 0)
    for n in (4096, 4096 * 8 * 3 + 4096):
        src = torch.randint(-2 ** 31, 2 ** 31 - 1, (n // 4,), dtype=torch.int32, device=dev)
        dst = torch.zeros(n // 16, dtype=torch.int32, device=dev)
        _hip.stream_ceiling(src, dst, torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize()
        q = src.view(-1, 4, 256)
        want = q[:, 0] ^ q[:, 1] ^ q[:, 2] ^ q[:, 3]
        assert torch.equal(dst.view(-1, 256), want)


def test_misaligned_device_views():
    """a contiguous device view whose base is not 16-B aligned (flat[4:4100]) is
    quantized correctly by quantize / quantize_packed / quantize_model_packed /
    quantize_model_device, and does not take its batch down with it."""
    dev = torch.device(DEV, 0)
    flat = rand_bf16((8192,), 77, 0.02).to(dev)
    views = {"mis": flat[4:4100], "mis2": flat[1:3073].view(3, 1024), "ok": flat[:4096]}
    assert views["mis"].data_ptr() % 16 != 0
    q = Q(bits=4, symmetric=False)
    packed = q.quantize_model_packed(dict(views))
    device = q.quantize_model_device(dict(views), packed=False)
    for name, v in views.items():
        ref = orc.quantize(v.cpu(), bits=4, group_size=128, symmetric=False)
        rows = 1 if v.dim() <= 1 else v.shape[0]
        for pk in (q.quantize_packed(v), packed[name]):
            assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"].reshape(rows, -1), 4, 0)), name
            assert torch.equal(pk["scales"].cpu(), ref["scales"]), name
        assert torch.equal(device[name]["tensor_q"].cpu(), ref["tensor_q"]), name
        assert torch.equal(q.quantize(v)["tensor_q"], ref["tensor_q"]), name
