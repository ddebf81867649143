"""Opt-in per-group clip search (scale_method="search", include/awq_hip.h awq_quantize_search).

No reference counterpart (the reference stores scale_method and never reads it,
awq.py:66,111-112; SURVEY.md §8a "parity unpinned"): the bar is
  * candidate 0 alone (alpha = 1) reproduces the reference RTN result bit-exactly
    (pinned through the golden fixtures),
  * the search never increases a group's squared dequantization error over RTN,
  * the HIP kernel equals oracle_quantize_search bit-for-bit (GPU tests).
"""
import ctypes

import pytest
import torch

import golden_io as gio
from oracle import awq_oracle as orc


def _group_err(x, res, gs):
    """Per-group sum of squared errors of the reference dequantize, float64 [rows, G]."""
    dq = orc.dequantize(res).double()
    xd = x.double()
    R = 1 if x.dim() <= 1 else x.shape[0]
    K = x.numel() // R
    G = -(-K // gs)
    d = torch.zeros(R, G * gs, dtype=torch.float64)
    d[:, :K] = ((xd - dq) ** 2).reshape(R, K)
    return d.reshape(R, G, gs).sum(-1)


# ---------------------------------------------------------------- CPU: oracle properties
@pytest.mark.parametrize("case", [c for c in gio.ok_cases() if c["params"].get("group_size", 128) <= 256][::7],
                         ids=lambda c: c["name"])
def test_single_candidate_is_rtn_golden(case):
    x = gio.case_input(case)
    p = case["params"]
    res = orc.quantize(x, bits=p.get("bits", 4), group_size=p.get("group_size", 128),
                       symmetric=p.get("symmetric", True), per_channel=p.get("per_channel", True), search=(20, 1))
    T = gio.tensors()
    assert torch.equal(res["tensor_q"], T[case["name"] + ".tensor_q"])
    assert torch.equal(res["zero_points"], T[case["name"] + ".zero_points"])
    assert gio.same_bits(res["scales"], T[case["name"] + ".scales"])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("bits", [4, 8])
def test_search_never_worse_than_rtn(dtype, sym, bits):
    g = torch.Generator().manual_seed(5 + bits + sym)
    x = (torch.randn(24, 640, generator=g) * 0.03).to(dtype)
    x[3, :50] *= 40                                              # outliers: clipping pays off
    rtn = orc.quantize(x, bits=bits, group_size=128, symmetric=sym)
    srch = orc.quantize(x, bits=bits, group_size=128, symmetric=sym, search=(20, 10))
    e0, e1 = _group_err(x, rtn, 128), _group_err(x, srch, 128)
    # the search's own metric is an fp32 tree sum; allow its rounding, nothing more
    assert bool((e1 <= e0 * (1 + 1e-5) + 1e-30).all())
    if bits == 4:
        assert e1.sum() < 0.97 * e0.sum()                        # and it does find better clips


def test_search_nan_groups_keep_rtn():
    x = (torch.randn(4, 256) * 0.1).to(torch.bfloat16)
    x[1, 5] = float("nan")
    x[2, 200] = float("inf")
    rtn = orc.quantize(x, bits=4, group_size=128, symmetric=False)
    srch = orc.quantize(x, bits=4, group_size=128, symmetric=False, search=(20, 10))
    for r, g in [(1, 0), (2, 1)]:
        assert gio.same_bits(srch["scales"][r, g], rtn["scales"][r, g])
        assert torch.equal(srch["tensor_q"][r, g * 128:(g + 1) * 128], rtn["tensor_q"][r, g * 128:(g + 1) * 128])


def test_search_validation():
    from awq_quantizer.quantization import AWQQuantizer
    q = AWQQuantizer(scale_method="search", logger_level="ERROR")
    assert q.search_candidates == 10
    assert AWQQuantizer(scale_method="mse", logger_level="ERROR").search_candidates == 0
    assert AWQQuantizer(scale_method="search", search_grid=4, search_max_shrink=1.0,
                        logger_level="ERROR").search_candidates == 4
    with pytest.raises(ValueError, match="search_grid"):
        AWQQuantizer(scale_method="search", search_grid=0, logger_level="ERROR")
    with pytest.raises(ValueError, match="search_max_shrink"):
        AWQQuantizer(scale_method="search", search_max_shrink=0.0, logger_level="ERROR")
    with pytest.raises(ValueError, match="Unsupported scale calibration method"):
        AWQQuantizer(scale_method="grid", logger_level="ERROR")


def test_cli_accepts_search():
    from awq_quantizer.main import parse_args
    a = parse_args(["--model_id", "m", "--output_dir", "o", "--scale_method", "search", "--search_grid", "10"])
    assert (a.scale_method, a.search_grid, a.search_max_shrink) == ("search", 10, 0.5)


# ---------------------------------------------------------------- GPU: kernel vs oracle
SEARCH_CASES = [(torch.bfloat16, (40, 1024), 128), (torch.float16, (32, 1024), 128), (torch.bfloat16, (50, 768), 128),
                (torch.float16, (77, 768), 128), (torch.bfloat16, (3, 1280), 128), (torch.bfloat16, (768,), 128),
                (torch.bfloat16, (7, 300), 128), (torch.float16, (33, 300), 128),
                (torch.float32, (17, 1000), 64), (torch.float64, (5, 777), 100), (torch.bfloat16, (3, 2, 50), 32),
                (torch.bfloat16, (10, 10), 128), (torch.bfloat16, (60,), 128), (torch.float16, (4, 4096), 256)]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,shape,gs", SEARCH_CASES, ids=str)
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("bits", [4, 8])
def test_search_gpu_vs_oracle(dtype, shape, gs, sym, bits):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer.quantization import AWQQuantizer
    g = torch.Generator().manual_seed(17 + bits)
    x = (torch.randn(*shape, generator=g) * 0.05).to(dtype)
    if x.dim() == 2 and x.shape[1] > 64:
        x[0, 3] = 2.0                                            # an outlier group
    q = AWQQuantizer(bits=bits, group_size=gs, symmetric=sym, scale_method="search", device="cuda",
                     logger_level="ERROR")
    ref = orc.quantize(x, bits=bits, group_size=gs, symmetric=sym, search=(20, 10))
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
    if x.numel() >= gs:
        pk = q.quantize_packed(x)
        assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], bits, q.qmin))
        assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], bits, q.qmin))


def test_search_group_size_limit():
    """One 8-element chunk per error slot, 64 slots: group_size <= 512."""
    from awq_quantizer import _hip
    lib = _hip.load_library()
    assert lib.awq_quantize_search(ctypes.c_void_p(16), 0, 4, 2048, 1024, 4, 0, 20, 10, None, None,
                                   ctypes.c_void_p(16), None, None, None) != 0
    assert "group_size <= 512" in _hip.last_error()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_search_gpu_fast_path_special_groups(dtype):
    """The streaming kernel's search on NaN / inf / constant / near-constant groups (fp16:
    a shrunk candidate of a near-constant group can hit the scale clamp min 0)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer.quantization import AWQQuantizer
    g = torch.Generator().manual_seed(8)
    x = (torch.randn(32, 1024, generator=g) * 0.05)
    x[0, 5] = float("nan")
    x[1, 200] = float("inf")
    x[2, :128] = 0.25
    x[3, 128:256] = 0.25
    x[3, 130] = 0.2502                     # near-constant: shrunk candidates collapse
    x[4, 256:384] = torch.linspace(-6e-5, 6e-5, 128)
    x[5, :128] = -3.0
    x = x.to(dtype)
    for sym in (False, True):
        q = AWQQuantizer(bits=4, symmetric=sym, scale_method="search", device="cuda", logger_level="ERROR")
        ref = orc.quantize(x, bits=4, group_size=128, symmetric=sym, search=(20, 10))
        res = q.quantize(x)
        assert torch.equal(res["tensor_q"], ref["tensor_q"])
        assert torch.equal(res["zero_points"], ref["zero_points"])
        assert gio.same_bits(res["scales"], ref["scales"])


@pytest.mark.gpu
@pytest.mark.parametrize("bits,sym", [(4, False), (4, True), (8, False), (8, True)])
def test_search_gpu_f16_packed_chain_mixed_scales(bits, sym):
    """Round 6: the fp16 search's packed chain (awq_fast.hip chunk_err_f16p, taken by waves whose
    candidate scales are all < 14) next to the Markstein chain (a wave with one scale >= 14) and
    the special path: small / large / near-constant large-magnitude (t overflows to inf) /
    subnormal groups, rows mixing them inside one wave, against the oracle bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer.quantization import AWQQuantizer
    g = torch.Generator().manual_seed(60 + bits + sym)
    R, K = 48, 4096
    x = torch.randn(R, K, generator=g) * 0.05
    x[4:8] *= 1000.0                                              # s >= 14: Markstein waves
    x[8:12] = 1000.0 + torch.randn(4, K, generator=g) * 0.3       # near-constant, large magnitude
    x[12:16] = 4000.0 + torch.randn(4, K, generator=g) * 2.0      # x / s beyond the fp16 range
    x[16:20] *= 2e-5                                              # subnormal fp16 values and scales
    x[20:24, 128 * 5:128 * 6] *= 600.0                            # one large group inside plain waves
    x[24:28, ::2] = torch.round(x[24:28, ::2] * 64) / 64          # coarse grid: quotient ties
    x[28, 300] = float("nan")
    x[29, 1000:1128] = 0.125                                      # constant group (s = 0)
    x = x.half()
    q = AWQQuantizer(bits=bits, group_size=128, symmetric=sym, scale_method="search", device="cuda",
                     logger_level="ERROR")
    ref = orc.quantize(x, bits=bits, group_size=128, symmetric=sym, search=(20, 10))
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
    pk = q.quantize_packed(x)
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], bits, q.qmin))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n_grid", [65536, 65537, 100000])
def test_search_gpu_large_grids_alpha(dtype, n_grid):
    """Round 6: alpha_i = (n - i) / n by one Markstein correction for n <= 65536 (exhaustively the
    IEEE quotient, verify_recip alpha) and by the IEEE division beyond — both sides of the switch
    against the oracle, with candidates whose shrink still moves bf16 / fp16 extremes."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer.quantization import AWQQuantizer
    g = torch.Generator().manual_seed(n_grid % 97)
    x = (torch.randn(16, 1024, generator=g) * 0.05).to(dtype)
    x[0, 3] = 2.0
    shrink = 300.0 / n_grid                     # 300 candidates: alpha down to ~0.995 .. 0.997
    q = AWQQuantizer(bits=4, group_size=128, symmetric=False, scale_method="search", search_grid=n_grid,
                     search_max_shrink=shrink, device="cuda", logger_level="ERROR")
    n_cand = min(n_grid, max(1, int(shrink * n_grid)))
    ref = orc.quantize(x, bits=4, group_size=128, symmetric=False, search=(n_grid, n_cand))
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])


@pytest.mark.gpu
def test_search_gpu_special_values_and_rtn_identity():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer.quantization import AWQQuantizer
    from test_gpu_parity import special_tensor
    x = special_tensor((32, 1024), 3)
    for sym in (False, True):
        ref = orc.quantize(x, bits=4, group_size=128, symmetric=sym, search=(16, 8))
        q = AWQQuantizer(bits=4, symmetric=sym, scale_method="search", search_grid=16, device="cuda",
                         logger_level="ERROR")
        res = q.quantize(x)
        assert torch.equal(res["tensor_q"], ref["tensor_q"])
        assert gio.same_bits(res["scales"], ref["scales"])
        one = AWQQuantizer(bits=4, symmetric=sym, scale_method="search", search_grid=16,
                           search_max_shrink=1 / 16, device="cuda", logger_level="ERROR").quantize(x)
        rtn = AWQQuantizer(bits=4, symmetric=sym, device="cuda", logger_level="ERROR").quantize(x)
        assert torch.equal(one["tensor_q"], rtn["tensor_q"])
        assert gio.same_bits(one["scales"], rtn["scales"])


@pytest.mark.gpu
def test_search_gpu_model_packed_routes_generic():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer.quantization import AWQQuantizer
    g = torch.Generator().manual_seed(2)
    ts = {"a": (torch.randn(64, 512, generator=g) * 0.02).bfloat16(), "b": (torch.randn(768, generator=g)).bfloat16()}
    q = AWQQuantizer(bits=4, symmetric=False, scale_method="search", device="cuda", logger_level="ERROR")
    out = q.quantize_model_packed(ts)
    for n, t in ts.items():
        ref = orc.quantize(t, bits=4, group_size=128, symmetric=False, search=(20, 10))
        rows = 1 if t.dim() == 1 else t.shape[0]
        assert torch.equal(out[n]["qweight"].cpu(), orc.pack_rows(ref["tensor_q"].reshape(rows, -1), 4, 0))
        assert gio.same_bits(out[n]["scales"].cpu(), ref["scales"])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("gs,bits,sym", [(128, 4, False), (64, 8, True), (32, 4, True), (256, 4, False)])
def test_search_ragged_launch_equals_per_tensor(dtype, gs, bits, sym):
    """Round 5: the clip search of a whole tensor set in ONE ragged launch
    (awq_quantize_ragged_search, PackedBatch(search=...), quantize_model_packed /
    quantize_model_device) gives the bits of the per-tensor search and of the oracle —
    many shapes incl. padded rows (K % gs != 0, K % 8 == 0), 1-D tensors and a NaN group."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer.quantization import AWQQuantizer
    g = torch.Generator().manual_seed(gs + bits)
    shapes = [(96, 1024), (1, 4096), (2048,), (33, 512), (7, 3 * gs), (5, gs * 2 + 8 * 3), (300, 256)]
    ts = {f"t{i}": (torch.randn(*s, generator=g) * 0.03).to(dtype) for i, s in enumerate(shapes)}
    ts["t0"][3, 17] = float("nan")
    ts["t4"][1, 5] = 1.5
    q = AWQQuantizer(bits=bits, group_size=gs, symmetric=sym, scale_method="search", device="cuda",
                     logger_level="ERROR")
    out = q.quantize_model_packed(ts)
    dev_out = q.quantize_model_device(ts, packed=False)
    assert sorted(out) == sorted(ts) == sorted(dev_out)
    for n, t in ts.items():
        ref = orc.quantize(t, bits=bits, group_size=gs, symmetric=sym, search=(20, 10))
        rows = 1 if t.dim() == 1 else t.shape[0]
        assert torch.equal(out[n]["qweight"].cpu(), orc.pack_rows(ref["tensor_q"].reshape(rows, -1), bits, q.qmin)), n
        assert torch.equal(out[n]["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], bits, q.qmin)), n
        assert gio.same_bits(out[n]["scales"].cpu(), ref["scales"]), n
        one = q.quantize_packed(t)
        assert torch.equal(one["qweight"], out[n]["qweight"]) and torch.equal(one["qzeros"], out[n]["qzeros"]), n
        assert torch.equal(dev_out[n]["tensor_q"].cpu(), ref["tensor_q"]), n
        assert gio.same_bits(dev_out[n]["scales"].cpu(), ref["scales"]), n
