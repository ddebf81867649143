"""Activation-aware per-input-channel scale search (scale_method="awq"; include/awq_hip.h
awq_act_*).

No reference counterpart (the reference collects no activations, awq.py:66 stores
scale_method and never reads it) and AutoAWQ is not installed: parity with either is
unpinned.  The bar here:
  * the HIP kernels equal oracle_act_* bit for bit from the same inputs only: statistics,
    w_mean, the scale table (its power function is defined as a fixed sequence of IEEE fp64
    ops both sides implement, include/awq_hip.h awq_pow — round 5; before, libm pow left it
    at 1 fp32 ulp and the tests fed the GPU's table to the oracle), per-group losses, loss
    totals, the chosen candidate, the scaled weight and its quantization;
  * properties: without duo scaling candidate 0 is the identity scaling, i.e. exactly the
    reference RTN result; the chosen candidate's loss is the minimum; on activations with
    outlier channels the search beats RTN on the weighted error.
"""
import ctypes
import math

import pytest
import torch

from oracle import awq_oracle as orc


def _layer(seed, rows=(96, 40), K=512, dtype=torch.bfloat16, outliers=True):
    g = torch.Generator().manual_seed(seed)
    ws = {f"w{i}": (torch.randn(r, K, generator=g) * 0.02).to(dtype) for i, r in enumerate(rows)}
    amp = torch.ones(K)
    if outliers:
        amp[torch.randperm(K, generator=g)[: K // 32]] = 30.0          # salient channels
    x = (torch.randn(300, K, generator=g) * amp).to(dtype)
    return ws, x


def _ulp_diff(a, b):
    ia = a.contiguous().view(torch.int32).to(torch.int64)
    ib = b.contiguous().view(torch.int32).to(torch.int64)
    return (ia - ib).abs()


# ---------------------------------------------------------------- CPU: oracle properties
def test_oracle_stats_match_fp64():
    ws, x = _layer(0, dtype=torch.bfloat16)
    xm, xs = orc.act_stats(x)
    xd = x.double()
    assert int(_ulp_diff(xm, (xd.abs().sum(0) / x.shape[0]).float()).max()) <= 1
    assert int(_ulp_diff(xs, ((xd * xd).sum(0) / x.shape[0]).float()).max()) <= 1


def test_oracle_det_pow_accuracy():
    """awq_pow (the table's power function) against libm pow: <= 2^-40 relative over every
    fp32 magnitude the statistics take (a definition, not pow itself: the table then
    differs from a libm-pow table in at most the last fp32 bit, on rare channels)."""
    import ctypes
    L = orc.lib()
    L.oracle_det_pow.restype = ctypes.c_double
    L.oracle_det_pow.argtypes = [ctypes.c_double, ctypes.c_double]
    g = torch.Generator().manual_seed(3)
    xs = torch.exp2(torch.rand(20000, generator=g, dtype=torch.float64) * 270 - 145).float().double()
    worst = 0.0
    for i, x in enumerate(xs.tolist()):
        r = (i % 65) / 64
        want = x ** r
        worst = max(worst, abs(L.oracle_det_pow(x, r) - want) / want)
    assert worst < 2 ** -40, worst
    assert L.oracle_det_pow(0.0, 0.0) == 1.0 and L.oracle_det_pow(0.0, 0.5) == 0.0
    assert L.oracle_det_pow(float("inf"), 0.5) == float("inf") and L.oracle_det_pow(float("nan"), 0.0) == 1.0


def test_oracle_table_formula():
    ws, x = _layer(1)
    xm, _ = orc.act_stats(x)
    wm = orc.weight_mean(list(ws.values()), 128)
    for duo in (False, True):
        t = orc.act_scale_table(xm, wm if duo else None, 10)
        for i in (0, 3, 9):
            r = i / 10
            raw = xm.double() ** r
            if duo:
                raw = raw / (wm.double() ** (1 - r) + 1e-4)
            raw = raw.clamp(min=1e-4)
            want = (raw / (raw.max() * raw.min()).sqrt()).float()
            assert int(_ulp_diff(t[i], want).max()) <= 1
    assert torch.equal(orc.act_scale_table(xm, None, 10)[0], torch.ones_like(xm))    # r = 0: identity


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_ratio0_without_duo_is_rtn(dtype):
    ws, x = _layer(2, dtype=dtype)
    r = orc.awq_search(list(ws.values()), x, n_grid=8, duo_scaling=False)
    for w in ws.values():
        s0 = orc.apply_input_scale(w, r["table"][0])
        assert torch.equal(s0.view(torch.uint8), w.contiguous().view(torch.uint8))
    # the weighted error of candidate 0 is the RTN error
    assert r["losses"][r["best"]] <= r["losses"][0]


def test_search_beats_rtn_on_salient_channels():
    ws, x = _layer(3, rows=(128,), K=1024)
    r = orc.awq_search(list(ws.values()), x, n_grid=20, duo_scaling=False)
    assert r["best"] > 0
    assert r["losses"][r["best"]] < 0.9 * r["losses"][0]
    # the diagonal loss IS the expected output error for independent channels: check it
    # against the true output MSE on the calibration set, best candidate vs RTN
    w = next(iter(ws.values()))
    xs = x.double()
    def out_err(res, s):
        dq = orc.dequantize(res).double() / s.double()
        return ((xs @ (dq - w.double()).t()) ** 2).mean()
    rtn = orc.quantize(w, bits=4, group_size=128, symmetric=False)
    assert out_err(r["results"][0], r["input_scale"]) < out_err(rtn, torch.ones(w.shape[1]))


def test_nan_weight_keeps_candidate_0():
    ws, x = _layer(4)
    w = next(iter(ws.values())).clone()
    w[3, 17] = float("nan")
    r = orc.awq_search([w], x, n_grid=6, duo_scaling=False)
    assert r["best"] == 0 and bool(torch.isnan(r["losses"]).all())


def test_quantizer_validation_without_gpu():
    from awq_quantizer.quantization import AWQQuantizer
    q = AWQQuantizer(scale_method="awq", logger_level="ERROR")
    assert q.duo_scaling and q.search_grid == 20
    with pytest.raises(ValueError, match="search_grid"):
        AWQQuantizer(scale_method="awq", search_grid=300, logger_level="ERROR")
    with pytest.raises(ValueError, match="2-D"):
        q.quantize_layer_group({"a": torch.zeros(128)})
    with pytest.raises(ValueError, match="share in_features"):
        q.quantize_layer_group({"a": torch.zeros(8, 128), "b": torch.zeros(8, 256)})
    with pytest.raises(ValueError, match="power-of-two"):
        AWQQuantizer(scale_method="awq", group_size=96, logger_level="ERROR").quantize_layer_group(
            {"a": torch.zeros(8, 192)})
    with pytest.raises(ValueError, match="scale_method='awq'"):
        AWQQuantizer(logger_level="ERROR").quantize_layer_group({"a": torch.zeros(8, 128)})


def test_capi_validation_without_gpu():
    from awq_quantizer import _hip
    lib = _hip.load_library()
    P = ctypes.c_void_p(16)
    assert lib.awq_act_scale_table(P, None, 128, 0, P, None) != 0
    assert "n_grid" in _hip.last_error()
    assert lib.awq_act_search_losses(P, 0, 8, 384, 96, 4, 0, P, None, 4, P, P, 24, None) != 0
    assert "power-of-two" in _hip.last_error()
    assert lib.awq_act_search_losses(P, 3, 8, 256, 128, 4, 0, P, None, 4, P, P, 16, None) != 0
    assert "bf16 / fp16 / fp32" in _hip.last_error()
    assert lib.awq_act_search_losses(P, 0, 8, 256, 128, 4, 0, P, None, 4, P, P, 15, None) != 0
    assert "part_stride" in _hip.last_error()
    assert lib.awq_act_stats(P, 0, 0, 128, P, P, P, None) != 0
    assert lib.awq_act_recip_table(P, 0, 128, P, None) != 0 and "n_grid" in _hip.last_error()


def _levels_sum(v, sizes):
    """fp64 sum of v in nested ascending levels (sizes innermost first), as include/awq_hip.h
    defines the canonical orders: [64, 16, 32] for the loss totals, [32, 8] for a column block."""
    import numpy as np
    v = np.asarray(v, dtype=np.float64)
    if not sizes:
        s = 0.0
        for t in v:
            s += t
        return s
    n = sizes[0]
    return _levels_sum([_levels_sum(v[i:i + n], []) for i in range(0, len(v), n)], sizes[1:])


def test_oracle_select_order():
    """The oracle's loss totals follow the header's four-level order (checked against an
    independent restatement on a part array spanning two super-blocks, magnitudes chosen so
    that the order changes the bits)."""
    g = torch.Generator().manual_seed(3)
    stride = 33 * 1024 + 517
    part = (torch.rand(3, stride, generator=g) * 10.0 ** torch.randint(-6, 6, (3, stride), generator=g)).float()
    losses, best = orc.act_search_select(part)
    for i in range(3):
        want = _levels_sum(part[i].double().numpy(), [64, 16, 32])
        assert losses[i].item() == want
    assert best == int(torch.argmin(losses))


def test_oracle_stats_order():
    g = torch.Generator().manual_seed(4)
    x = (torch.randn(300, 5, generator=g) * 10.0 ** torch.randint(-4, 4, (300, 5), generator=g)).float()
    xm, xs = orc.act_stats(x)
    xd = x.double().numpy()
    for k in range(5):
        blocks = [_levels_sum(abs(xd[b:b + 256, k]), [32]) for b in (0, 256)]
        assert xm[k].item() == float(torch.tensor(_levels_sum(blocks, []) / 300).float())
        blocks = [_levels_sum(xd[b:b + 256, k] ** 2, [32]) for b in (0, 256)]
        assert xs[k].item() == float(torch.tensor(_levels_sum(blocks, []) / 300).float())


# ---------------------------------------------------------------- GPU: kernels vs oracle
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("T", [1, 255, 300, 1024])
def test_gpu_stats_bit_exact(dtype, T):
    dev = _gpu()
    from awq_quantizer import _hip
    g = torch.Generator().manual_seed(T)
    x = (torch.randn(T, 777, generator=g) * 3).to(dtype)
    x[0, 5] = float("inf")
    xm, xs = _hip.act_stats(x.to(dev))
    om, os_ = orc.act_stats(x)
    assert torch.equal(xm.cpu().view(torch.int32), om.view(torch.int32))
    assert torch.equal(xs.cpu().view(torch.int32), os_.view(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("gs", [8, 32, 64, 128, 256, 512])
@pytest.mark.parametrize("special", [False, True])
@pytest.mark.parametrize("K", [1024, 1280])
def test_gpu_weight_mean_bit_exact(dtype, gs, special, K):
    """gs 32 / 64 / 128 / 256 take the one-pass kernel, 8 / 512 the two-pass path; 300 rows
    = a full 256-row block + a partial one (partial stage and sub-block); K 1280: a partial
    column tile; special: NaN and inf groups."""
    dev = _gpu()
    from awq_quantizer import _hip
    if K % gs:
        pytest.skip("K % gs != 0")
    g = torch.Generator().manual_seed(gs)
    ws = [(torch.randn(r, K, generator=g) * 0.05).to(dtype) for r in (300, 1, 17, 600)]
    ws[1][0, :gs] = 0.0                                            # an all-zero group
    if special:
        ws[0][5, 3] = float("nan")
        ws[2][3, 700] = float("inf")
        ws[3][599, K - 24] = float("-inf")
    got = _hip.weight_mean([w.to(dev) for w in ws], gs).cpu()
    assert torch.equal(got.view(torch.int32), orc.weight_mean(ws, gs).view(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("gs", [8, 32, 128])
def test_gpu_weight_mean_wide_range_bit_exact(dtype, gs):
    """Weights spanning the dtype's whole finite range (subnormals, |w| < 2^-60 next to normal
    group maxima, group maxima > 2^60, zeros) against the oracle's division."""
    dev = _gpu()
    from awq_quantizer import _hip
    g = torch.Generator().manual_seed(gs)
    lo, hi = {torch.bfloat16: (-133, 127), torch.float16: (-24, 15), torch.float32: (-149, 127)}[dtype]
    e = torch.rand(300, 1024, generator=g, dtype=torch.float64) * (hi - lo) + lo
    sign = torch.where(torch.rand(300, 1024, generator=g) < 0.5, -1.0, 1.0).double()
    w = (sign * torch.exp2(e)).to(dtype)
    w[7, :gs] = 0.0
    w[8, :gs] = torch.tensor(2.0 ** (lo + 2), dtype=torch.float64).to(dtype)
    w[9, 1] = torch.tensor(2.0 ** -70).to(dtype) if dtype != torch.float16 else 0.0
    got = _hip.weight_mean([w.to(dev)], gs).cpu()
    assert torch.equal(got.view(torch.int32), orc.weight_mean([w], gs).view(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("duo", [False, True])
@pytest.mark.parametrize("n_grid,K", [(20, 2048), (64, 4096), (7, 384)])
def test_gpu_table_bit_exact(duo, n_grid, K):
    """The scale table from the same x_mean / w_mean: GPU == oracle bit for bit (awq_pow)."""
    dev = _gpu()
    from awq_quantizer import _hip
    ws, x = _layer(5, K=K)
    xm, _ = orc.act_stats(x)
    wm = orc.weight_mean(list(ws.values()), 128) if duo else None
    t = _hip.act_scale_table(xm.to(dev), None if wm is None else wm.to(dev), n_grid).cpu()
    o = orc.act_scale_table(xm, wm, n_grid)
    assert torch.equal(t.view(torch.int32), o.view(torch.int32))


@pytest.mark.gpu
def test_gpu_table_wide_range_bit_exact():
    """Statistics across the whole fp32 range (subnormal, tiny, huge, zero, inf, NaN) and
    n_grid 256: every power the table takes, bit for bit."""
    dev = _gpu()
    from awq_quantizer import _hip
    g = torch.Generator().manual_seed(77)
    xm = torch.exp2(torch.rand(4096, generator=g, dtype=torch.float64) * 250 - 140).float()
    wm = torch.exp2(torch.rand(4096, generator=g, dtype=torch.float64) * 250 - 140).float()
    xm[:6] = torch.tensor([0.0, 1e-45, 1e-40, 3e38, 1.0, 2.0])
    for duo in (False, True):
        o = orc.act_scale_table(xm, wm if duo else None, 256)
        for ws_ in (True, False):   # awq_act_scale_table_ws and awq_act_scale_table
            t = _hip.act_scale_table(xm.to(dev), wm.to(dev) if duo else None, 256, workspace=ws_).cpu()
            assert torch.equal(t.view(torch.int32), o.view(torch.int32)), ws_
    bad = xm.clone()
    bad[7], bad[8] = float("inf"), float("nan")
    for ws_ in (True, False):
        t = _hip.act_scale_table(bad.to(dev), wm.to(dev), 16, workspace=ws_).cpu()
        assert torch.equal(t.view(torch.int32), orc.act_scale_table(bad, wm, 16).view(torch.int32)), ws_


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 255, 256, 257, 14336])
def test_gpu_table_workspace_slices(K):
    """awq_act_scale_table_ws at slice edges (256 channels per workgroup) == the oracle and
    the workspace-free kernel."""
    dev = _gpu()
    from awq_quantizer import _hip
    g = torch.Generator().manual_seed(K)
    xm = torch.exp2(torch.rand(K, generator=g) * 20 - 10)
    wm = torch.exp2(torch.rand(K, generator=g) * 20 - 10)
    for duo in (False, True):
        o = orc.act_scale_table(xm, wm if duo else None, 20)
        a = _hip.act_scale_table(xm.to(dev), wm.to(dev) if duo else None, 20).cpu()
        b = _hip.act_scale_table(xm.to(dev), wm.to(dev) if duo else None, 20, workspace=False).cpu()
        assert torch.equal(a.view(torch.int32), o.view(torch.int32))
        assert torch.equal(b.view(torch.int32), o.view(torch.int32))


LOSS_CASES = [(torch.bfloat16, 128, 4, False), (torch.bfloat16, 128, 4, True), (torch.bfloat16, 128, 8, False),
              (torch.float16, 128, 4, False), (torch.float16, 64, 4, True), (torch.float32, 128, 4, False),
              (torch.bfloat16, 32, 4, False), (torch.bfloat16, 512, 4, False), (torch.bfloat16, 8, 8, True),
              (torch.float16, 256, 8, False), (torch.float32, 32, 8, True), (torch.float16, 32, 4, False),
              (torch.bfloat16, 256, 4, True), (torch.float32, 64, 4, True), (torch.bfloat16, 16, 4, False),
              (torch.float32, 256, 4, False)]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,gs,bits,sym", LOSS_CASES, ids=str)
def test_gpu_losses_bit_exact(dtype, gs, bits, sym):
    dev = _gpu()
    from awq_quantizer import _hip
    ws, x = _layer(6 + gs + bits, rows=(70, 5, 33), K=1024, dtype=dtype)
    wl = list(ws.values())
    xm, xs = orc.act_stats(x)
    table = _hip.act_scale_table(xm.to(dev), _hip.weight_mean([w.to(dev) for w in wl], gs), 12)
    part = _hip.act_search_losses([w.to(dev) for w in wl], xs.to(dev), table, gs, bits, sym)
    losses, best, s_best = _hip.act_search_select(part, table)
    ol, ob, opart = orc.act_search_losses(wl, xs, table.cpu(), gs, bits, sym)
    assert torch.equal(part.cpu().view(torch.int32), opart.view(torch.int32))
    assert torch.equal(losses.cpu().view(torch.int64), ol.view(torch.int64))
    assert int(best.item()) == ob
    assert torch.equal(s_best.cpu(), table.cpu()[ob])


@pytest.mark.gpu
@pytest.mark.parametrize("bits,sym", [(4, False), (4, True), (8, False)])
def test_gpu_losses_f16_packed_mixed_scales(bits, sym):
    """Round 6: the fp16 loss path in packed fp16 (AWQ_ACT_F16_PACKED: w' pairs, the plain
    quotient in waves whose scales are all < 14, the Markstein one otherwise, t + z as
    v_pk_add_f16) — rows of small, large (s >= 14), near-constant large-magnitude, subnormal and
    overflowing (w * s beyond the fp16 range) weights, a NaN, a constant group; the partial losses
    against the oracle bit for bit."""
    dev = _gpu()
    from awq_quantizer import _hip
    g = torch.Generator().manual_seed(90 + bits + sym)
    K = 1024
    w = torch.randn(72, K, generator=g) * 0.02
    w[8:16] *= 3000.0                                            # s >= 14 groups
    w[16:24] = 900.0 + torch.randn(8, K, generator=g) * 0.5      # near-constant, large magnitude
    w[24:32] = 50000.0 + torch.randn(8, K, generator=g) * 30.0   # w * s overflows fp16 for s > ~1.31
    w[32:40] *= 1e-4                                             # subnormal fp16 weights
    w[40:48, 128 * 2:128 * 3] *= 5000.0                          # one large group in a small row
    w[48:56, ::2] = torch.round(w[48:56, ::2] * 256) / 256        # coarse grid: ties
    w[60, 7] = float("nan")
    w[61, 256:384] = 0.5                                         # constant group
    w = w.half()
    amp = torch.ones(K)
    amp[torch.randperm(K, generator=g)[: K // 32]] = 30.0
    x = (torch.randn(200, K, generator=g) * amp).half()
    xm, xs = orc.act_stats(x)
    table = _hip.act_scale_table(xm.to(dev), _hip.weight_mean([w.to(dev)], 128), 12)
    part = _hip.act_search_losses([w.to(dev)], xs.to(dev), table, 128, bits, sym)
    _, _, opart = orc.act_search_losses([w], xs, table.cpu(), 128, bits, sym)
    assert torch.equal(part.cpu().view(torch.int32), opart.view(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("n_grid", [1, 2, 3])
@pytest.mark.parametrize("dtype,gs", [(torch.bfloat16, 128), (torch.float16, 256), (torch.bfloat16, 32)], ids=str)
def test_gpu_losses_short_grids(n_grid, dtype, gs):
    """The loss kernel's LDS table ring at its edges: one, two and three candidates (the
    first slot's wait, the harmless reload after the last candidate), two DMAs per candidate
    (gs 256) and partial DMAs (gs 32), rows that leave row blocks partly empty."""
    dev = _gpu()
    from awq_quantizer import _hip
    ws, x = _layer(40 + n_grid + gs, rows=(37, 8), K=512, dtype=dtype)
    wl = list(ws.values())
    xm, xs = orc.act_stats(x)
    table = _hip.act_scale_table(xm.to(dev), None, n_grid)
    part = _hip.act_search_losses([w.to(dev) for w in wl], xs.to(dev), table, gs, 4, False)
    _, _, opart = orc.act_search_losses(wl, xs, table.cpu(), gs, 4, False)
    assert torch.equal(part.cpu().view(torch.int32), opart.view(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("n_grid,stride", [(1, 1), (5, 1023), (7, 64 * 1024 + 100), (20, 917504),
                                           (256, 40 * 1024), (64, 3200 * 1024)], ids=str)
def test_gpu_select_bit_exact(n_grid, stride):
    """awq_act_search_select on part arrays of every shape class: partial sub-blocks, one
    block, several super-blocks (a Llama-3-8B gate/up group list: 917 504 groups), the
    maximum grid, and candidate batches (n_grid x super-blocks beyond one LDS batch)."""
    dev = _gpu()
    from awq_quantizer import _hip
    g = torch.Generator(device=dev).manual_seed(n_grid)
    part = torch.rand(n_grid, stride, generator=g, device=dev)
    part *= torch.exp2(torch.randint(-20, 20, (n_grid, stride), generator=g, device=dev).float())
    table = torch.rand(n_grid, 64, generator=g, device=dev)
    losses, best, s_best = _hip.act_search_select(part, table)
    ol, ob = orc.act_search_select(part)
    assert torch.equal(losses.cpu().view(torch.int64), ol.view(torch.int64))
    assert int(best.item()) == ob and torch.equal(s_best.cpu(), table.cpu()[ob])


@pytest.mark.gpu
@pytest.mark.parametrize("T", [31, 32, 33, 257, 4096])
def test_gpu_stats_sub_blocks(T):
    """Sub-block edges (32 tokens) and many blocks; K % 8 != 0 takes the per-column kernel."""
    dev = _gpu()
    from awq_quantizer import _hip
    g = torch.Generator().manual_seed(T)
    for K in (64, 100):
        x = (torch.randn(T, K, generator=g) * torch.exp2(torch.randint(-10, 10, (T, K), generator=g).float()))
        x = x.bfloat16()
        xm, xs = _hip.act_stats(x.to(dev))
        om, os_ = orc.act_stats(x)
        assert torch.equal(xm.cpu().view(torch.int32), om.view(torch.int32))
        assert torch.equal(xs.cpu().view(torch.int32), os_.view(torch.int32))


@pytest.mark.gpu
def test_selftest_markstein_quotient_exhaustive():
    """The loss kernel's fp32(dq / s) from RN(1/s) + one Markstein correction == the IEEE
    division for every s in [1, 2) and every positive finite fp16 dq (2.7e11 pairs; by scale
    invariance this covers the whole range awq_act_recip_table enables)."""
    from awq_quantizer import _hip
    assert _hip.selftest(1, _gpu()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32], ids=str)
def test_gpu_losses_rtable_paths_agree(dtype):
    """Markstein path (rtable) == IEEE path (no rtable) bit for bit, including a table whose
    channels leave the proven range for part of the candidates (those waves fall back)."""
    dev = _gpu()
    from awq_quantizer import _hip
    ws, x = _layer(21, rows=(64, 33), K=1024, dtype=dtype)
    wl = [w.to(dev) for w in ws.values()]
    xm, xs = orc.act_stats(x)
    table = _hip.act_scale_table(xm.to(dev), None, 10)
    table[3, 100] = 2.0 ** -70                 # outside [2^-60, 2^60]: IEEE fallback for those waves
    table[7, 900] = 2.0 ** 70
    rt = _hip.act_recip_table(table)
    # outside the range: NaN (round 6; a quotient through it is NaN and its wave redoes the
    # candidate with IEEE divisions)
    assert math.isnan(float(rt[3, 100])) and math.isnan(float(rt[7, 900]))
    assert torch.equal(rt.cpu()[:3], torch.ones(()) / table.cpu()[:3])      # IEEE fp32 1/s (CPU)
    a = _hip.act_search_losses(wl, xs.to(dev), table, 128, 4, False, rtable=rt)
    b = _hip.act_search_losses(wl, xs.to(dev), table, 128, 4, False, use_rtable=False)
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    _, _, opart = orc.act_search_losses([w.cpu() for w in wl], xs, table.cpu(), 128, 4, False)
    # (fp16: the 2^70 channel overflows to inf, its groups' losses are NaN; NaN payloads are
    # not part of the definition, so NaN positions are compared and the rest bit for bit)
    a = a.cpu()
    assert torch.equal(torch.isnan(a), torch.isnan(opart))
    assert torch.equal(torch.where(torch.isnan(a), 0, a).view(torch.int32),
                       torch.where(torch.isnan(opart), 0, opart).view(torch.int32))


@pytest.mark.gpu
def test_gpu_losses_special_values():
    dev = _gpu()
    from awq_quantizer import _hip
    ws, x = _layer(9, rows=(40,), K=512)
    w = ws["w0"].clone()
    w[1, :128] = 0.0                     # all-zero group
    w[2, 128:256] = 1e-30                # constant tiny group (bf16 subnormal range)
    w[3, 5] = 3e38                       # overflows once scaled
    xm, xs = orc.act_stats(x)
    table = _hip.act_scale_table(xm.to(dev), None, 8)
    part = _hip.act_search_losses([w.to(dev)], xs.to(dev), table, 128, 4, False)
    _, _, opart = orc.act_search_losses([w], xs, table.cpu(), 128, 4, False)
    a, b = part.cpu(), opart
    assert torch.equal(torch.isnan(a), torch.isnan(b))
    assert torch.equal(torch.where(torch.isnan(a), 0, a).view(torch.int32), torch.where(torch.isnan(b), 0, b).view(torch.int32))
    w[7, 9] = float("nan")
    part = _hip.act_search_losses([w.to(dev)], xs.to(dev), table, 128, 4, False)
    losses, best, _ = _hip.act_search_select(part, table)
    assert int(best.item()) == 0 and bool(torch.isnan(losses.cpu()).all())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_gpu_apply_input_scale_bit_exact(dtype):
    dev = _gpu()
    from awq_quantizer import _hip
    ws, x = _layer(10, rows=(33,), K=640, dtype=dtype)
    w = ws["w0"]
    s = torch.rand(640) * 4 + 0.01
    got = _hip.apply_input_scale(w.to(dev), s.to(dev)).cpu()
    assert torch.equal(got.view(torch.uint8), orc.apply_input_scale(w, s).view(torch.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("duo", [False, True])
@pytest.mark.parametrize("dtype,sym", [(torch.bfloat16, False), (torch.float16, True), (torch.float32, False)])
def test_gpu_quantize_layer_group_end_to_end(dtype, sym, duo):
    dev = _gpu()
    from awq_quantizer.quantization import AWQQuantizer
    ws, x = _layer(11, rows=(128, 64, 64), K=1024, dtype=dtype)
    q = AWQQuantizer(bits=4, group_size=128, symmetric=sym, scale_method="awq", duo_scaling=duo, device="cuda",
                     logger_level="ERROR")
    out = q.quantize_layer_group(ws, x.to(dev))
    ref = orc.awq_search(list(ws.values()), x, n_grid=20, symmetric=sym, duo_scaling=duo)   # oracle from the inputs alone
    assert torch.equal(out["table"].cpu().view(torch.int32), ref["table"].view(torch.int32))
    assert out["best"] == ref["best"]
    assert torch.equal(out["losses"].cpu().view(torch.int64), ref["losses"].view(torch.int64))
    assert torch.equal(out["input_scale"].cpu(), ref["input_scale"])
    for (name, r), rr in zip(out["results"].items(), ref["results"]):
        rows = ws[name].shape[0]
        assert torch.equal(r["qweight"].cpu(), orc.pack_rows(rr["tensor_q"].reshape(rows, -1), 4, q.qmin)), name
        assert torch.equal(r["qzeros"].cpu(), orc.pack_rows(rr["zero_points"], 4, q.qmin)), name
        assert torch.equal(r["scales"].cpu().view(torch.int16), rr["scales"].view(torch.int16)), name
        assert r["input_scale"] is out["input_scale"]
    # unpacked (reference-format) results of the same search
    out2 = q.quantize_layer_group(ws, x_mean=ref["x_mean"], x_sq=ref["x_sq"], packed=False)
    for (name, r), rr in zip(out2["results"].items(), ref["results"]):
        assert torch.equal(r["tensor_q"].cpu(), rr["tensor_q"]), name


@pytest.mark.gpu
def test_gpu_ratio0_is_rtn():
    dev = _gpu()
    from awq_quantizer.quantization import AWQQuantizer
    ws, x = _layer(12, rows=(64,), K=512)
    q = AWQQuantizer(bits=4, symmetric=False, scale_method="awq", search_grid=1, duo_scaling=False, device="cuda",
                     logger_level="ERROR")
    out = q.quantize_layer_group(ws, x.to(dev))
    rtn = AWQQuantizer(bits=4, symmetric=False, device="cuda", logger_level="ERROR").quantize_packed(ws["w0"])
    assert out["best"] == 0
    assert torch.equal(out["results"]["w0"]["qweight"], rtn["qweight"])
    assert torch.equal(out["input_scale"].cpu(), torch.ones(512))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32], ids=str)
@pytest.mark.parametrize("gs", [32, 64, 128, 256])
@pytest.mark.parametrize("bits,sym", [(4, False), (4, True), (8, False)])
@pytest.mark.parametrize("shape", [(70, 1024), (9, 3072), (33, 4096), (5, 512)], ids=str)
def test_gpu_quantize_groups_scaled_equals_two_step(dtype, gs, bits, sym, shape):
    """awq_quantize_groups_scaled == awq_apply_input_scale into a copy + awq_quantize_groups,
    bit for bit: tiles inside one row (K 4096), spanning two rows (K 3072) and many rows
    (K 512 / 1024: the modulo path), special values in W and in s (0, huge -> inf products,
    NaN)."""
    dev = _gpu()
    from awq_quantizer import _hip
    R, K = shape
    if K % gs:
        pytest.skip("K % gs != 0")
    g = torch.Generator().manual_seed(R * K + gs + bits)
    w = (torch.randn(R, K, generator=g) * 0.05).to(dtype)
    w[0, 5] = float("nan")
    w[R - 1, K - 3] = float("inf")
    s = torch.exp2(torch.randn(K, generator=g) * 3)
    s[7], s[K - 1] = 0.0, 3e38
    if K > 40:
        s[40] = float("nan")
    w, s = w.to(dev), s.to(dev)
    G, per = K // gs, 32 // bits

    def outs():
        return (torch.full((R, -(-K // per)), -1, dtype=torch.int32, device=dev),
                torch.full((R, -(-G // per)), -1, dtype=torch.int32, device=dev),
                torch.full((R, G), 0x7BCD, dtype=torch.int16, device=dev).view(torch.float16))
    a, b = outs(), outs()
    _hip.quantize_groups_scaled(w, s, gs, bits, sym, qweight=a[0], qzeros=a[1], scales=a[2])
    sw = _hip.apply_input_scale(w, s)
    kw = {}
    if not _hip.packs_directly(dtype, R, K, gs):
        kw = dict(tensor_q=torch.empty(R * K, dtype=torch.int32, device=dev),
                  zeros=torch.empty(R, G, dtype=torch.int32, device=dev))
    _hip.quantize_groups(sw, R, K, gs, bits, sym, qweight=b[0], qzeros=b[1], scales=b[2], **kw)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert torch.equal(a[2].view(torch.int16), b[2].view(torch.int16))


@pytest.mark.gpu
def test_gpu_layer_group_one_pass_equals_scaled_copy():
    """quantize_layer_group's one-pass path == quantize_packed of the scaled weights."""
    dev = _gpu()
    from awq_quantizer import _hip
    from awq_quantizer.quantization import AWQQuantizer
    ws, x = _layer(91, rows=(96, 40), K=1024)
    q = AWQQuantizer(bits=4, group_size=128, symmetric=False, scale_method="awq", search_grid=10, device="cuda",
                     logger_level="ERROR")
    res = q.quantize_layer_group({k: v.to(dev) for k, v in ws.items()}, x.to(dev))
    for name, w in ws.items():
        ref = q.quantize_packed(_hip.apply_input_scale(w.to(dev), res["input_scale"]))
        got = res["results"][name]
        for k in ("qweight", "qzeros"):
            assert torch.equal(got[k], ref[k]), (name, k)
        assert torch.equal(got["scales"].view(torch.int16), ref["scales"].view(torch.int16))
