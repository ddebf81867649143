"""Every BASELINE.json config quantized bit-exactly on the GPU against the oracle
(VERDICT r1 "configs untested"; reference src/awq_quantizer/quantization/awq.py:286-374
for the arithmetic, main.py:216-330 for the CLI flow).

  * opt-125m: the whole 196-tensor set in ONE ragged launch (the bench's step), parity
    mode — every tensor_q / zero_points / scales / qweight / qzeros compared in full;
  * opt-350m: a multi-file safetensors checkpoint of the exact shape manifest streamed
    through the CLI (reader pool -> pinned staging -> H2D -> ragged launches -> D2H ->
    chunk writer), every written result compared in full;
  * Llama-3-70B: one tensor of each distinct shape (the 28672x8192 MLP, the
    128256x8192 embedding, ...) in one ragged launch, packed outputs compared in full
    (Llama-3-8B's shapes: tests/test_gpu_parity.py::test_full_size_properties).

Synthetic N(0, 0.02) bf16 weights (no checkpoints offline)."""
import json
import os
import sys

import pytest
import torch

import golden_io as gio
from oracle import awq_oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import bench  # noqa: E402  (shape manifests + the bench's synthetic data generator)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awq_quantizer import _hip
    _hip.require_device(torch.device("cuda", 0))


def _check_full(name, x, out, bits, sym, parity):
    qmin = orc.qrange(bits, sym)[0]
    ref = orc.quantize(x.cpu(), bits=bits, group_size=128, symmetric=sym)
    rows = 1 if x.dim() <= 1 else x.shape[0]
    tq = ref["tensor_q"].reshape(rows, -1)
    assert torch.equal(out["qweight"].cpu(), orc.pack_rows(tq, bits, qmin)), name
    assert torch.equal(out["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], bits, qmin)), name
    assert gio.same_bits(out["scales"].cpu(), ref["scales"]), name
    if parity:
        assert torch.equal(out["tensor_q"].cpu().reshape(rows, -1), tq), name
        assert torch.equal(out["zero_points"].cpu(), ref["zero_points"]), name


@pytest.mark.parametrize("bits,sym", [(4, False), (4, True), (8, False)], ids=str)
def test_opt125m_whole_set_one_launch(bits, sym):
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device("cuda", 0)
    shapes = bench.shapes_of("opt-125m")
    assert len(shapes) == 196
    inputs = bench.make_set(shapes, 7 + bits + sym, dev)
    b = PackedBatch(inputs, bits=bits, symmetric=sym, parity=True)
    b.run()
    torch.cuda.synchronize()
    res = b.results()
    assert sorted(res) == sorted(inputs)
    for name, x in inputs.items():
        _check_full(name, x, res[name], bits, sym, parity=True)


def test_llama3_70b_distinct_shapes_full():
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device("cuda", 0)
    shapes = [s for s, _ in bench.WORKLOADS["llama3-70b"]]
    inputs = bench.make_set(shapes, 70, dev)
    b = PackedBatch(inputs, bits=4, symmetric=False)
    b.run()
    torch.cuda.synchronize()
    res = b.results()
    for name, x in inputs.items():
        _check_full(name, x, res[name], 4, False, parity=False)


@pytest.mark.parametrize("fmt", ["reference", "packed"])
def test_opt350m_streamed_through_cli(tmp_path, fmt):
    """The opt-350m manifest (388 tensors, 662 MB bf16) as a 3-file safetensors checkpoint,
    quantized by the CLI with the reference defaults (4-bit asym, gs 128); every result
    read back through metadata.json equals the oracle."""
    from safetensors.torch import save_file
    from awq_quantizer.main import main
    shapes = bench.shapes_of("opt-350m")
    assert len(shapes) == 388
    cpu = bench.make_set(shapes, 350, torch.device("cpu"))
    names = list(cpu)
    d = tmp_path / "model"
    d.mkdir()
    per = -(-len(names) // 3)
    for i in range(3):
        save_file({n: cpu[n] for n in names[i * per:(i + 1) * per]}, str(d / f"model-{i + 1:05d}-of-00003.safetensors"))
    out = tmp_path / "out"
    assert main(["--model_id", str(d), "--output_dir", str(out), "--log_level", "ERROR",
                 "--output_format", fmt]) == 0
    meta = json.load(open(out / "metadata.json"))
    assert meta["num_tensors"] == 388 and sorted(meta["tensor_to_chunk"]) == sorted(names)
    sizes = [cpu[n].numel() for n in meta["tensor_to_chunk"]]
    assert sizes == sorted(sizes, reverse=True)                      # processing order, main.py:259
    chunks = {}
    for name, c in meta["tensor_to_chunk"].items():
        if c not in chunks:
            chunks = {c: torch.load(str(out / f"model_chunk_{c:04d}.pt"), weights_only=True)}
        r = chunks[c][name]
        x = cpu[name]
        ref = orc.quantize(x, bits=4, group_size=128, symmetric=False)
        if fmt == "reference":
            assert torch.equal(r["tensor_q"], ref["tensor_q"]), name
            assert torch.equal(r["zero_points"], ref["zero_points"]), name
            assert gio.same_bits(r["scales"], ref["scales"]), name
            assert (int(r["bits"]), int(r["group_size"]), bool(r["symmetric"])) == (4, 128, False)
        else:
            rows = 1 if x.dim() <= 1 else x.shape[0]
            assert torch.equal(r["qweight"], orc.pack_rows(ref["tensor_q"].reshape(rows, -1), 4, 0)), name
            assert torch.equal(r["qzeros"], orc.pack_rows(ref["zero_points"], 4, 0)), name
            assert gio.same_bits(r["scales"], ref["scales"]), name
