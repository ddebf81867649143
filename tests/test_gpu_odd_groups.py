"""4-bit tensors whose rows hold an odd number of groups (G = K / gs odd: Qwen2.5-0.5B's
hidden size 896 = 7 groups of 128, K = 3200 = 25 groups, ...) on the streaming kernel.

Their rows' zero points do not fill whole qzeros bytes, so they take word tiles: whole
qzeros words per tile (whole rows when G <= 32 / bits), every word produced inside one
tile (awq_internal.h).  The values follow the reference's per-group arithmetic
(awq.py:173-213, 286-374); the qzeros layout is north_star's packing (`orc.pack_rows`).
Bit-exact against the oracle, independent of what the output buffers held before the
launch, and stable over repeats.
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


def rand(shape, seed, scale=0.02, dtype=torch.bfloat16, dev="cpu"):
    g = torch.Generator(device=dev).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=dev) * scale).to(dtype)


def batch(inputs, gs, sym=False, parity=False):
    from awq_quantizer.quantization.batch import PackedBatch
    return PackedBatch(inputs, bits=4, symmetric=sym, parity=parity, group_size=gs)


def check_batch(b, inputs, gs, sym):
    qmin = -8 if sym else 0
    for name, res in b.results().items():
        x = inputs[name].cpu()
        rows = 1 if x.dim() == 1 else x.shape[0]
        ref = orc.quantize(x, bits=4, group_size=gs, symmetric=sym)
        assert torch.equal(res["qzeros"].cpu(), orc.pack_rows(ref["zero_points"].reshape(rows, -1), 4, qmin)), name
        assert torch.equal(res["qweight"].cpu(), orc.pack_rows(ref["tensor_q"].reshape(rows, -1), 4, qmin)), name
        assert gio.same_bits(res["scales"].cpu(), ref["scales"].reshape(rows, -1)), name


def odd_shapes(gs):
    # G = 1, 3, 5, 7, 9, 25, 33 with row counts that put straddles at many tile offsets
    return [(37, gs), (29, 3 * gs), (23, 5 * gs), (61, 7 * gs), (17, 9 * gs), (13, 25 * gs), (7, 33 * gs),
            (7 * gs,), (3, 5, 7 * gs)]


@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32], ids=["bf16", "f16", "f32"])
@pytest.mark.parametrize("gs", [32, 64, 128, 256])
def test_odd_groups_vs_oracle(gs, dtype, sym):
    dev = torch.device(DEV, 0)
    inputs = {f"t{i}": rand(s, 70 * gs + 5 * i + sym, 0.02, dtype).to(dev) for i, s in enumerate(odd_shapes(gs))}
    for fill in (0, -1):             # no output word may depend on the old contents
        b = batch(inputs, gs, sym)
        for o in b.out.values():
            o["qzeros"].fill_(fill)
        b.run()
        torch.cuda.synchronize()
        check_batch(b, inputs, gs, sym)


@pytest.mark.parametrize("sym", [False, True])
def test_odd_groups_parity_mode_and_single(sym):
    """Single-tensor API and the reference-layout outputs for K = 896 (G = 7)."""
    from awq_quantizer.quantization import AWQQuantizer
    q = AWQQuantizer(bits=4, group_size=128, symmetric=sym, device=DEV, logger_level="ERROR")
    x = rand((300, 896), 896 + sym, 1.0)
    x[3, :128] = float("nan")
    x[5, 128:256] = 0.0
    x[8, 768:] = 1e-6
    ref = orc.quantize(x, bits=4, group_size=128, symmetric=sym)
    res = q.quantize(x)
    assert torch.equal(res["tensor_q"], ref["tensor_q"])
    assert torch.equal(res["zero_points"], ref["zero_points"])
    assert gio.same_bits(res["scales"], ref["scales"])
    pk = q.quantize_packed(x)
    assert torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], 4, q.qmin))
    assert torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], 4, q.qmin))


def test_odd_groups_full_size_embedding():
    """Qwen2.5-0.5B's embedding shape (151936 x 896, G = 7, 1.06 M groups): packed outputs
    == oracle over the whole tensor, and three launches into garbage-filled outputs give
    identical bytes."""
    dev = torch.device(DEV, 0)
    x = rand((151936, 896), 5, 0.02, torch.bfloat16, dev)
    b = batch({"emb": x}, 128)
    outs = []
    for fill in (0, -1, 0x5A5A5A5A):
        for t in b.out["emb"].values():   # raw bit patterns (scales: int16 view)
            (t if t.dtype == torch.int32 else t.view(torch.int16)).fill_(fill if t.dtype == torch.int32 else fill & 0x7FFF)
        b.run()
        torch.cuda.synchronize()
        outs.append({k: v.clone() for k, v in b.out["emb"].items()})
    for o in outs[1:]:
        for k in o:
            assert torch.equal(o[k], outs[0][k]), k
    ref = orc.quantize(x.cpu(), bits=4, group_size=128, symmetric=False)
    assert torch.equal(outs[0]["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], 4, 0))
    assert torch.equal(outs[0]["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], 4, 0))
    assert gio.same_bits(outs[0]["scales"].cpu(), ref["scales"])
