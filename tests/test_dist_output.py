"""torchrun-mode output of the CLI on CPU (gloo, world 2 / 3; the GPU box runs the same
code over RCCL): per-rank chunk files, the gather-to-rank-0 option,
the AutoAWQ shards, and the failure agreement (a rank that fails as a whole makes every
rank exit 1 instead of leaving the others blocked in a collective).

The quantize pipeline itself needs the GPU, so the workers replace
`awq_quantizer.main.quantize_stream` with a fake that returns deterministic result dicts
(same contract: results into `out`, every tensor reported to `on_done`); everything after
it — chunk numbering, renames, metadata.json, shard index, agreement — is the product
code.  Bar: the union of the per-rank files, loaded through metadata.json (or the shard
index), equals what the single-process writer produces from the same results (reference
layout, src/awq_quantizer/main.py:430-512)."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
from safetensors.torch import load_file, save_file

FAIL_NAMES = {"model.layers.3.mlp.weight", "model.layers.11.mlp.weight"}


def _model(tmp_path):
    d = tmp_path / "model"
    d.mkdir()
    g = torch.Generator().manual_seed(0)
    t = {f"model.layers.{i}.mlp.weight": (torch.randn(8 * (i % 7 + 1), 128, generator=g) * 0.02).bfloat16()
         for i in range(23)}
    t["model.norm.weight"] = torch.ones(128, dtype=torch.bfloat16)
    t["model.embed_tokens.weight"] = torch.randn(64, 128, generator=g).bfloat16()
    t["model.small"] = torch.randn(10, 10, generator=g).bfloat16()
    t["model.int"] = torch.arange(300, dtype=torch.int32)
    names = list(t)
    save_file({n: t[n] for n in names[:13]}, str(d / "model-00001-of-00002.safetensors"))
    save_file({n: t[n] for n in names[13:]}, str(d / "model-00002-of-00002.safetensors"))
    return str(d), t


def fake_result(name, fmt, shape=(3, 16)):
    h = sum(map(ord, name)) % 1000
    if fmt == "sized":      # packed fields at the tensor's own packed shapes, random bits
        import zlib
        rows = shape[0] if len(shape) > 1 else 1
        K = int(torch.Size(shape).numel()) // rows
        G = -(-K // 128)
        g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
        rnd = lambda *sh: torch.randint(-2 ** 31, 2 ** 31 - 1, sh, generator=g, dtype=torch.int64).to(torch.int32)
        return {"qweight": rnd(rows, -(-K // 8)), "qzeros": rnd(rows, -(-G // 8)),
                "scales": (rnd(rows, G) >> 16).to(torch.int16).view(torch.float16),
                "bits": torch.tensor(4, dtype=torch.int32), "group_size": torch.tensor(128, dtype=torch.int32),
                "symmetric": torch.tensor(False), "shape": torch.tensor(list(shape), dtype=torch.int64)}
    if fmt == "autoawq":
        return {"qweight": torch.full((128, 1), h, dtype=torch.int32), "qzeros": torch.full((1, 1), h, dtype=torch.int32),
                "scales": torch.full((1, 8), h / 1000, dtype=torch.float16)}
    r = {"qweight": torch.full((3, 2), h, dtype=torch.int32), "qzeros": torch.full((3, 1), -h, dtype=torch.int32),
         "scales": torch.full((3, 1), h / 1000, dtype=torch.float16), "bits": torch.tensor(4, dtype=torch.int32),
         "group_size": torch.tensor(128, dtype=torch.int32), "symmetric": torch.tensor(False),
         "shape": torch.tensor(list(shape), dtype=torch.int64)}
    return r


def _fake_stream(fmt, fail_rank, rank):
    def quantize_stream(loader, infos, quantizer, device, readers, lookahead, packed, out, lock, logger,
                        memory_efficient=False, keep_on_device=False, batch_bytes=0, export_autoawq=False,
                        act_stats=None, on_done=None, **_):
        for k, info in enumerate(infos):
            if rank == fail_rank and k == 1:
                raise RuntimeError("device lost (injected)")
            if info.name in FAIL_NAMES:
                if on_done:
                    on_done(info.name, None)
                continue
            r = fake_result(info.name, "autoawq" if export_autoawq else fmt, tuple(info.shape))
            with lock:
                out.update({info.name: r})
            if on_done:
                on_done(info.name, r)
    return quantize_stream


def _worker(rank, world, port, model_dir, out_dir, fmt, extra, fail_rank, q, inject=""):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), AWQ_DIST_BACKEND="gloo")
    if isinstance(out_dir, list):      # per-rank directories: not one shared output directory
        out_dir = out_dir[rank]
    try:
        from awq_quantizer import main as M
        M.quantize_stream = _fake_stream(fmt, fail_rank, rank)
        if inject == "meta" and rank == 0:          # the last commit step fails after the renames
            def bad_meta(*a, **k):
                raise OSError("disk full (injected)")
            M._write_metadata = bad_meta
        rc = M.main(["--model_id", model_dir, "--output_dir", out_dir, "--log_level", "CRITICAL", "--chunk_size", "4",
                     "--output_format", "packed" if fmt == "sized" else fmt] + extra)
        q.put((rank, rc))
    except BaseException as e:  # surface to the parent
        q.put((rank, repr(e)))
        raise


def _run(world, model_dir, out_dir, fmt="packed", extra=(), fail_rank=-1, inject=""):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, world, port, model_dir, out_dir, fmt, list(extra), fail_rank, q,
                                               inject))
             for r in range(world)]
    for p in procs:
        p.start()
    rcs = dict(q.get(timeout=150) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    return [rcs[r] for r in range(world)]


def _load_chunks(d):
    meta = json.load(open(os.path.join(d, "metadata.json")))
    out = {}
    for name, c in meta["tensor_to_chunk"].items():
        ext = ".safetensors" if meta["format"] == "safetensors" else ".pt"
        path = os.path.join(d, f"model_chunk_{c:04d}{ext}")
        if ext == ".pt":
            out[name] = torch.load(path, weights_only=True)[name]
        else:
            flat = load_file(path)
            out[name] = {k[len(name) + 1:]: v for k, v in flat.items() if k.startswith(name + ".")}
    return meta, out


def _single_process_files(tmp_path, model_dir, fmt, st):
    """What the single-process writer makes of the same results."""
    from awq_quantizer.main import save_model_in_chunks, select_tensors
    from awq_quantizer.model_loading import load_model_from_path
    index = load_model_from_path(model_dir, logger_level="ERROR").tensor_index()
    sel = select_tensors(index)
    ordered = [i.name for i in sel]
    res = {i.name: fake_result(i.name, fmt, tuple(i.shape)) for i in sel if i.name not in FAIL_NAMES}
    d = str(tmp_path / "single")
    save_model_in_chunks(res, d, chunk_size=4, use_safetensors=st)
    return d, ordered


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,st", [(2, False), (3, False), (2, True)])
def test_per_rank_chunks_load_like_single_process(tmp_path, world, st):
    model_dir, _ = _model(tmp_path)
    out = str(tmp_path / "out")
    extra = ["--save_safetensors"] if st else []
    assert _run(world, model_dir, out, "packed", extra) == [0] * world
    ref_dir, ordered = _single_process_files(tmp_path, model_dir, "packed", st)
    meta, got = _load_chunks(out)
    ref_meta, want = _load_chunks(ref_dir)
    # tensor_to_chunk: every successful tensor, processing order (bytes descending, main.py:259)
    assert list(meta["tensor_to_chunk"]) == list(ref_meta["tensor_to_chunk"]) == \
        [n for n in ordered if n not in FAIL_NAMES]
    for k in ("chunk_size", "format", "num_tensors", "quantization_params"):
        assert meta[k] == ref_meta[k], k
    assert set(got) == set(want)
    for n in want:
        assert list(got[n]) == list(want[n]) and all(torch.equal(got[n][f], want[n][f]) for f in want[n]), n
    # global chunk numbers 0..num_chunks-1, each file written by one rank, no temporaries left
    ext = ".safetensors" if st else ".pt"
    files = sorted(f for f in os.listdir(out) if f != "metadata.json")
    assert files == [f"model_chunk_{c:04d}{ext}" for c in range(meta["num_chunks"])]
    assert sorted(set(meta["tensor_to_chunk"].values())) == list(range(meta["num_chunks"]))
    assert max(list(meta["tensor_to_chunk"].values()).count(c) for c in range(meta["num_chunks"])) <= 4


@pytest.mark.timeout(300)
def test_gather_mode_writes_single_process_layout(tmp_path):
    model_dir, _ = _model(tmp_path)
    out = str(tmp_path / "out")
    assert _run(2, model_dir, out, "packed", ["--dist_output", "gather"]) == [0, 0]
    ref_dir, _ = _single_process_files(tmp_path, model_dir, "packed", False)
    meta, got = _load_chunks(out)
    ref_meta, want = _load_chunks(ref_dir)
    assert meta == ref_meta                         # the same chunk grouping: rank 0 wrote everything
    for n in want:
        assert all(torch.equal(got[n][f], want[n][f]) for f in want[n]), n


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["per_rank", "gather"])
def test_failed_rank_fails_every_rank(tmp_path, mode):
    """a rank whose pipeline raises must not leave the others blocked in a
    collective; every rank exits 1 and nothing is published."""
    model_dir, _ = _model(tmp_path)
    out = str(tmp_path / "out")
    assert _run(2, model_dir, out, "packed", ["--dist_output", mode], fail_rank=1) == [1, 1]
    assert not os.path.exists(os.path.join(out, "metadata.json"))
    assert [f for f in os.listdir(out) if "chunk" in f] == []


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [1, 2, 3])
def test_autoawq_shards_and_failed_linears(tmp_path, world):
    """AutoAWQ output: per-rank shards + model.safetensors.index.json (world 1: the
    single-process model.safetensors); linear weights that failed to quantize are copied
    unquantized and listed in modules_to_not_convert."""
    from awq_quantizer.main import is_linear_weight
    from awq_quantizer.model_loading import load_model_from_path
    model_dir, src = _model(tmp_path)
    with open(os.path.join(model_dir, "config.json"), "w") as f:
        json.dump({"model_type": "llama"}, f)
    out = str(tmp_path / "out")
    if world == 1:
        from awq_quantizer import main as M
        saved = M.quantize_stream
        M.quantize_stream = _fake_stream("autoawq", -1, 0)
        try:
            assert M.main(["--model_id", model_dir, "--output_dir", out, "--log_level", "CRITICAL",
                           "--output_format", "autoawq"]) == 0
        finally:
            M.quantize_stream = saved
        got = load_file(os.path.join(out, "model.safetensors"))
    else:
        assert _run(world, model_dir, out, "autoawq") == [0] * world
        index = json.load(open(os.path.join(out, "model.safetensors.index.json")))
        files = sorted(set(index["weight_map"].values()))
        assert files == [f"model-{k + 1:05d}-of-{len(files):05d}.safetensors" for k in range(len(files))]
        got = {}
        for f in files:
            part = load_file(os.path.join(out, f))
            assert sorted(k for k, v in index["weight_map"].items() if v == f) == sorted(part)
            got.update(part)
        assert index["metadata"]["total_size"] == sum(v.numel() * v.element_size() for v in got.values())
    infos = load_model_from_path(model_dir, logger_level="ERROR").tensor_index()
    linear = {i.name for i in infos if i.numel >= 128 and is_linear_weight(i, 128)}
    want = {}
    for n, t in src.items():
        if n in linear and n not in FAIL_NAMES:
            r = fake_result(n, "autoawq")
            for f in ("qweight", "qzeros", "scales"):
                want[f"{n[:-len('.weight')]}.{f}"] = r[f]
        else:
            want[n] = t
    assert sorted(got) == sorted(want)
    assert all(torch.equal(got[k], want[k]) for k in want)
    qc = json.load(open(os.path.join(out, "quant_config.json")))
    cfg = json.load(open(os.path.join(out, "config.json")))
    nc = sorted(n[: -len(".weight")] for n in FAIL_NAMES)
    assert sorted(qc["modules_to_not_convert"]) == nc
    assert sorted(cfg["quantization_config"]["modules_to_not_convert"]) == nc


@pytest.mark.timeout(300)
def test_per_rank_falls_back_to_gather_without_a_shared_directory(tmp_path):
    """per-rank chunk files are only a checkpoint if every rank writes into the
    directory rank 0's metadata.json describes.  Ranks that do not see one shared output
    directory (node-local disks) fall back to the gather layout: rank 0 writes everything."""
    model_dir, _ = _model(tmp_path)
    outs = [str(tmp_path / "out0"), str(tmp_path / "out1")]
    assert _run(2, model_dir, outs, "packed") == [0, 0]
    ref_dir, _ = _single_process_files(tmp_path, model_dir, "packed", False)
    meta, got = _load_chunks(outs[0])
    ref_meta, want = _load_chunks(ref_dir)
    assert meta == ref_meta
    for n in want:
        assert all(torch.equal(got[n][f], want[n][f]) for f in want[n]), n
    assert not os.path.exists(outs[1]) or [f for f in os.listdir(outs[1]) if "chunk" in f or "shared" in f] == []
    assert [f for f in os.listdir(outs[0]) if f.startswith(".awq_shared")] == []


@pytest.mark.timeout(300)
def test_failure_after_renames_unpublishes_every_chunk(tmp_path):
    """when the commit fails after the ranks renamed their chunks to global names
    (rank 0 cannot write metadata.json), every rank removes what it wrote: nothing stays."""
    model_dir, _ = _model(tmp_path)
    out = str(tmp_path / "out")
    assert _run(2, model_dir, out, "packed", inject="meta") == [1, 1]
    assert not os.path.exists(os.path.join(out, "metadata.json"))
    assert [f for f in os.listdir(out) if "chunk" in f] == []


def _llama70b_scaled_model(tmp_path):
    """The Llama-3-70B tensor set (723 names, tests/test_distributed.py) with rows / 256 and
    row lengths / 64, so byte sizes keep the real set's ratios (2-D) and order."""
    from test_distributed import _llama70b_names_shapes
    d = tmp_path / "model70b"
    d.mkdir()
    ts = _llama70b_names_shapes()
    g = torch.Generator().manual_seed(0)
    t = {n: (torch.randn(*((sh[0] // 256, sh[1] // 64) if len(sh) > 1 else (sh[0] // 64,)), generator=g) * 0.02)
         .bfloat16() for n, sh in ts.items()}
    names = list(t)
    for k in range(4):      # four shard files, like a real multi-file checkpoint
        save_file({n: t[n] for n in names[k::4]}, str(d / f"model-{k + 1:05d}-of-00004.safetensors"))
    return str(d)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["per_rank", "gather"])
def test_world8_llama70b_per_rank_chunks(tmp_path, mode):
    """the per-rank chunk commit at world 8 on the 70B ownership map (723
    names, the scaled set's LPT shard): the union of the 8 ranks' renumbered chunk files,
    read through metadata.json, is byte-exact against the single-process writer's files."""
    model_dir = _llama70b_scaled_model(tmp_path)
    out = str(tmp_path / "out")
    assert _run(8, model_dir, out, "sized", ["--dist_output", mode]) == [0] * 8
    from awq_quantizer.main import save_model_in_chunks, select_tensors
    from awq_quantizer.model_loading import load_model_from_path
    sel = select_tensors(load_model_from_path(model_dir, logger_level="ERROR").tensor_index())
    assert len(sel) == 723
    res = {i.name: fake_result(i.name, "sized", tuple(i.shape)) for i in sel if i.name not in FAIL_NAMES}
    ref = str(tmp_path / "single")
    save_model_in_chunks(res, ref, chunk_size=4)
    meta, got = _load_chunks(out)
    ref_meta, want = _load_chunks(ref)
    # every tensor, processing order; per-rank chunks of <= 4, numbered 0.. over the ranks
    assert list(meta["tensor_to_chunk"]) == list(ref_meta["tensor_to_chunk"]) == [i.name for i in sel]
    for k in ("chunk_size", "format", "num_tensors", "quantization_params"):
        assert meta[k] == ref_meta[k], k
    if mode == "gather":        # rank 0 wrote everything: the single-process grouping
        assert meta == ref_meta
    files = sorted(f for f in os.listdir(out) if f != "metadata.json")
    assert files == [f"model_chunk_{c:04d}.pt" for c in range(meta["num_chunks"])]
    assert max(list(meta["tensor_to_chunk"].values()).count(c) for c in range(meta["num_chunks"])) <= 4
    for n in want:
        assert list(got[n]) == list(want[n]), n
        for f in want[n]:
            a, b = got[n][f], want[n][f]
            assert a.dtype == b.dtype and a.shape == b.shape, (n, f)
            assert torch.equal(a.view(torch.int16) if a.dtype == torch.float16 else a,
                               b.view(torch.int16) if b.dtype == torch.float16 else b), (n, f)
