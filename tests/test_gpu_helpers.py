"""Measurement helpers of the C ABI on the GPU (include/awq_hip.h): awq_dequant_ceiling, the
1 : 8 read : write structure scripts/dq_ceiling_bench.py quotes dequantize_packed against,
writes the nibble expansion of its input (so the timed stream is real work, checked here)."""
import pytest
import torch


@pytest.mark.gpu
@pytest.mark.parametrize("n_out", [16, 4096, 1 << 20, (1 << 20) + 48])
def test_dequant_ceiling_writes_nibbles(n_out):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer import _hip
    dev = torch.device("cuda", 0)
    _hip.require_device(dev)
    quads = n_out // 4                      # fp32 outputs in groups of 4 (one 16-B store)
    g = torch.Generator().manual_seed(n_out)
    words = torch.randint(-2 ** 31, 2 ** 31 - 1, (-(-quads // 2),), generator=g, dtype=torch.int64).to(torch.int32)
    out = torch.full((n_out,), -1.0, dtype=torch.float32, device=dev)
    _hip.dequant_ceiling(words.to(dev), out, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    w = words.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    q = torch.arange(quads)
    half = (w[q // 2] >> (16 * (q % 2))) & 0xFFFF
    want = torch.stack([((half >> (4 * j)) & 15).float() for j in range(4)], dim=1).reshape(-1)
    assert torch.equal(out.cpu(), want)
