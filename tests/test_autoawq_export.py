"""AutoAWQ "GEMM" layout export (include/awq_hip.h
awq_export_autoawq_gemm).  Parity unpinned by the reference (it has no packed format) and
by AutoAWQ itself (not installed): checked against oracle.autoawq_pack, a restatement of
AutoAWQ's published packing, and by value (unpacking the export reproduces the reference
integers, dequantizing it reproduces the reference dequantize)."""
import ctypes

import pytest
import torch

import golden_io as gio
from oracle import awq_oracle as orc


def test_oracle_pack_roundtrip_and_order():
    g = torch.Generator().manual_seed(1)
    iw = torch.randint(0, 16, (40, 384), generator=g)
    z = torch.randint(0, 16, (40, 3), generator=g)
    sc = torch.rand(40, 3, generator=g).half()
    qw, qz, st = orc.autoawq_pack(iw, z, sc)
    assert qw.shape == (384, 5) and qz.shape == (3, 5) and st.shape == (3, 40)
    a, b = orc.autoawq_unpack(qw, qz)
    assert torch.equal(a, iw.t()) and torch.equal(b, z.t()) and torch.equal(st, sc.t())
    # nibble i of word c holds column 8c + AWQ_ORDER[i]
    one = torch.zeros(8, 1, dtype=torch.int64)
    one[2, 0] = 5
    w, _, _ = orc.autoawq_pack(one, torch.zeros(8, 1, dtype=torch.int64), torch.zeros(8, 1).half())
    assert int(w[0, 0]) == 5 << (4 * orc.AWQ_ORDER.index(2))


def test_export_validation_without_gpu():
    from awq_quantizer import _hip
    lib = _hip.load_library()
    assert lib.awq_export_autoawq_gemm(None, None, None, 64, 256, 128, 8, None, None, None, None) != 0
    assert "4-bit" in _hip.last_error()
    assert lib.awq_export_autoawq_gemm(None, None, None, 60, 256, 128, 4, None, None, None, None) != 0
    assert "% 8" in _hip.last_error()
    assert lib.awq_export_autoawq_gemm(None, None, None, 64, 200, 128, 4, None, None, None, None) != 0


CASES = [((64, 256), 128, False), ((72, 384), 128, True), ((128, 4096), 128, False), ((8, 128), 128, False),
         ((200, 768), 64, False), ((96, 1280), 128, True),
         # v2 qweight tiles are 256 x 256 nibbles: ragged n and k tiles, N/8 not a multiple of 4
         ((296, 2304), 128, False), ((520, 8192), 128, True), ((776, 512), 64, False), ((136, 5120), 128, False),
         # K % 32 != 0: the 4-B-load tile path
         ((24, 264), 8, False), ((40, 2072), 8, True)]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape,gs,sym", CASES, ids=str)
def test_export_matches_autoawq_packing(shape, gs, sym, dtype):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer.quantization import AWQQuantizer
    g = torch.Generator().manual_seed(shape[0] + shape[1])
    x = (torch.randn(*shape, generator=g) * 0.02).to(dtype)
    q = AWQQuantizer(bits=4, group_size=gs, symmetric=sym, device="cuda", logger_level="ERROR")
    ref = orc.quantize(x, bits=4, group_size=gs, symmetric=sym)
    ex = q.export_autoawq(q.quantize_packed(x))
    iw = ref["tensor_q"].to(torch.int64) - q.qmin              # unsigned fields
    zz = ref["zero_points"].to(torch.int64) - q.qmin
    qw, qz, st = orc.autoawq_pack(iw, zz, ref["scales"])
    assert torch.equal(ex["qweight"].cpu(), qw)
    assert torch.equal(ex["qzeros"].cpu(), qz)
    assert gio.same_bits(ex["scales"].cpu(), st)
    # AutoAWQ-style dequantization of the export == the reference dequantize, transposed
    a, b = orc.autoawq_unpack(ex["qweight"].cpu(), ex["qzeros"].cpu())
    zfull = b.repeat_interleave(gs, dim=0)
    sfull = ex["scales"].cpu().float().repeat_interleave(gs, dim=0)
    diff = (a - zfull).to(torch.float16)
    dq = (diff * sfull.to(torch.float16)).float()
    assert gio.same_bits(dq.t().contiguous(), orc.dequantize(ref))


@pytest.mark.gpu
def test_export_rejects_8bit_and_3d():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer.quantization import AWQQuantizer
    q8 = AWQQuantizer(bits=8, symmetric=False, device="cuda", logger_level="ERROR")
    with pytest.raises(RuntimeError, match="4-bit"):
        q8.export_autoawq(q8.quantize_packed(torch.randn(64, 256).bfloat16()))
    q = AWQQuantizer(bits=4, device="cuda", logger_level="ERROR")
    with pytest.raises(ValueError, match="2-D"):
        q.export_autoawq(q.quantize_packed(torch.randn(8, 2, 128).bfloat16()))


def _torch_autoawq_layout(qweight, qzeros, scales, N, K, G):
    """The AutoAWQ GEMM layout of row-major packed words, restated with torch tensor ops on
    the device (unpack nibbles, transpose, AWQ_ORDER interleave, repack)."""
    order = torch.tensor([0, 2, 4, 6, 1, 3, 5, 7], device=qweight.device)
    sh = 4 * torch.arange(8, device=qweight.device, dtype=torch.int64)

    def unpack(w, cols):
        return ((w.to(torch.int64).unsqueeze(-1) >> sh) & 15).reshape(w.shape[0], -1)[:, :cols]

    def pack(v):                                   # [R, C] nibbles -> [R, C / 8] AWQ_ORDER words
        v8 = v.reshape(v.shape[0], -1, 8)[:, :, order]
        x = (v8 << sh).sum(-1)
        return torch.where(x >= 2 ** 31, x - 2 ** 32, x).to(torch.int32)

    return (pack(unpack(qweight, K).t().contiguous()), pack(unpack(qzeros, G).t().contiguous()),
            scales.t().contiguous())


@pytest.mark.gpu
@pytest.mark.parametrize("N,K,gs", [(32768, 8192, 128), (32776, 8200, 40)], ids=str)
def test_export_large_nontemporal_path(N, K, gs):
    """qweight exports of >= 128 MB take the nontemporal-store kernel (csrc/awq_export.hip
    AWQ_EXPORT_NT_MIN): random packed words against the torch restatement of the layout.
    The second shape is ragged in both tile dimensions and takes the 4-B-load path."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer.quantization import AWQQuantizer
    dev = torch.device("cuda", 0)
    G = K // gs
    g = torch.Generator(device=dev).manual_seed(N + K)
    info = torch.iinfo(torch.int32)
    pk = {"qweight": torch.randint(info.min, info.max, (N, K // 8), generator=g, device=dev, dtype=torch.int32),
          "qzeros": torch.randint(info.min, info.max, (N, (G + 7) // 8), generator=g, device=dev, dtype=torch.int32),
          "scales": torch.randn(N, G, generator=g, device=dev).half(),
          "shape": torch.tensor([N, K]), "group_size": torch.tensor(gs), "bits": torch.tensor(4)}
    assert N * K // 2 >= 128 << 20
    q = AWQQuantizer(bits=4, group_size=gs, symmetric=False, device="cuda", logger_level="ERROR")
    ex = q.export_autoawq(pk)
    qw, qz, st = _torch_autoawq_layout(pk["qweight"], pk["qzeros"], pk["scales"], N, K, G)
    assert torch.equal(ex["qweight"], qw)
    assert torch.equal(ex["qzeros"], qz)
    assert torch.equal(ex["scales"].view(torch.int16), st.view(torch.int16))
