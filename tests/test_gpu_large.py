"""Tensors beyond 2^31 elements (> 4 GiB of bf16): every index and byte offset in the kernels
and the C ABI must be 64-bit.  Size-independent property (rows are independent,
awq.py:286-374): the whole tensor quantized in one call == its row blocks quantized one
call each, bit for bit; the same for dequantize_packed and for the ragged one-launch path
(quantize_model_packed) with a small tensor beside the big one.  The row blocks themselves
are < 2^31 elements and pinned against the oracle by the rest of the suite."""
import pytest
import torch

import golden_io as gio
from oracle import awq_oracle as orc

R, K = 132_000, 16_384          # 2 162 688 000 elements > 2^31
BLOCK = 16_500                  # rows per slice (270 M elements)


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda", 0)


def _big(dtype, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.empty(R, K, dtype=dtype, device=dev)
    for r0 in range(0, R, BLOCK):   # generate in slices: no fp32 temporary of the whole tensor
        x[r0:r0 + BLOCK] = (torch.randn(min(BLOCK, R - r0), K, device=dev, generator=g) * 0.02).to(dtype)
    x[7, :300] = 0.0                                     # a constant group
    x[R - 1, K - 200:] = float("nan")                  # NaN groups in the last row
    return x


def _outs(rows, G, dev, bits=4, fill=-0x5A5A5A5A):
    """Outputs pre-filled with a sentinel (different per call site): equal results mean both
    calls wrote them."""
    per = 32 // bits
    return (torch.full((rows, -(-K // per)), fill, dtype=torch.int32, device=dev),
            torch.full((rows, -(-G // per)), fill, dtype=torch.int32, device=dev),
            torch.full((rows, G), fill & 0x7FFF, dtype=torch.int16, device=dev).view(torch.float16))


def _oracle_rows(x, qw, qz, sc, r0, r1, gs):
    """Rows r0:r1 of the device result against the CPU oracle (awq.py restatement)."""
    ref = orc.quantize(x[r0:r1].cpu(), bits=4, group_size=gs, symmetric=False)
    assert torch.equal(qw[r0:r1].cpu(), orc.pack_rows(ref["tensor_q"], 4, 0)), (r0, r1)
    assert torch.equal(qz[r0:r1].cpu(), orc.pack_rows(ref["zero_points"], 4, 0)), (r0, r1)
    assert gio.same_bits(sc[r0:r1].cpu(), ref["scales"]), (r0, r1)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,gs", [(torch.bfloat16, 128), (torch.bfloat16, 100), (torch.float16, 64),
                                      (torch.float32, 128)], ids=str)
def test_gpu_beyond_2g_elements_equals_row_blocks(dtype, gs):
    dev = _gpu()
    from awq_quantizer import _hip
    assert R * K > 2 ** 31
    if not _hip.packs_directly(dtype, R, K, gs):
        pytest.skip("path needs int32 staging (tensor_q of the whole tensor)")
    x = _big(dtype, dev)
    G = -(-K // gs)
    qw, qz, sc = _outs(R, G, dev)
    _hip.quantize_groups(x, R, K, gs, 4, False, qweight=qw, qzeros=qz, scales=sc)
    # rows around element 2^31 (row 131 072) and the last rows (NaN groups) vs the oracle
    _oracle_rows(x, qw, qz, sc, 131_040, 131_104, gs)
    _oracle_rows(x, qw, qz, sc, R - 32, R, gs)
    for r0 in range(0, R, BLOCK):
        n = min(BLOCK, R - r0)
        bw, bz, bs = _outs(n, G, dev, fill=0x3C3C3C3C)
        _hip.quantize_groups(x[r0:r0 + n], n, K, gs, 4, False, qweight=bw, qzeros=bz, scales=bs)
        assert torch.equal(qw[r0:r0 + n], bw), r0
        assert torch.equal(qz[r0:r0 + n], bz), r0
        assert torch.equal(sc[r0:r0 + n].view(torch.int16), bs.view(torch.int16)), r0
    if dtype == torch.bfloat16 and gs == 128:
        del x
        out = torch.full((R, K), 7.0, dtype=torch.float32, device=dev)       # 8.6 GB
        _hip.dequantize_packed(qw, qz, sc, R, K, gs, 4, False, out)
        for r0 in range(0, R, 4 * BLOCK):
            n = min(4 * BLOCK, R - r0)
            part = torch.full((n, K), -1.0, dtype=torch.float32, device=dev)
            _hip.dequantize_packed(qw[r0:r0 + n], qz[r0:r0 + n], sc[r0:r0 + n], n, K, gs, 4, False, part)
            assert torch.equal(out[r0:r0 + n].view(torch.int32), part.view(torch.int32)), r0
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_beyond_2g_elements_ragged_launch():
    """quantize_model_packed: the big tensor and a small one in one ragged launch == the
    single-tensor call."""
    dev = _gpu()
    from awq_quantizer import _hip
    from awq_quantizer.quantization import AWQQuantizer
    x = _big(torch.bfloat16, dev, seed=1)
    small = (torch.randn(64, 4096, device=dev) * 0.02).bfloat16()
    q = AWQQuantizer(bits=4, group_size=128, symmetric=False, device="cuda", logger_level="ERROR")
    res = q.quantize_model_packed({"big": x, "small": small})
    G = K // 128
    qw, qz, sc = _outs(R, G, dev)
    _hip.quantize_groups(x, R, K, 128, 4, False, qweight=qw, qzeros=qz, scales=sc)
    _oracle_rows(x, qw, qz, sc, 131_040, 131_104, 128)
    big = res["big"]
    assert torch.equal(big["qweight"].to(dev), qw)
    assert torch.equal(big["qzeros"].to(dev), qz)
    assert torch.equal(big["scales"].to(dev).view(torch.int16), sc.view(torch.int16))
    one = q.quantize_packed(small)
    assert torch.equal(res["small"]["qweight"].to(dev), one["qweight"].to(dev))
