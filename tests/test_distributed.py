"""N>1 path on CPU: world_size-2 gloo process group (the bench/CLI use RCCL on the GPUs;
the logic under test — sharding, max-over-ranks timing, gather of packed shards to rank
0 — is backend-independent)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from awq_quantizer import distributed as D


def test_shard_lpt_deterministic_and_balanced():
    sizes = [100, 1, 50, 50, 49, 3, 3, 200, 7]
    own = D.shard(sizes, 3)
    assert own == D.shard(list(sizes), 3)
    loads = [sum(s for s, o in zip(sizes, own) if o == r) for r in range(3)]
    assert sum(loads) == sum(sizes) and max(loads) - min(loads) <= max(sizes)
    assert D.shard(sizes, 1) == [0] * len(sizes)
    # Llama-3-70B manifest over 8 ranks: imbalance < 1 %
    import bench
    shapes = bench.shapes_of("llama3-70b")
    sz = [int(torch.Size(s).numel()) * 2 for s in shapes]
    own = D.shard(sz, 8)
    loads = [sum(s for s, o in zip(sz, own) if o == r) for r in range(8)]
    assert max(loads) / min(loads) < 1.01


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, _, w = D.init("gloo")
        assert (r, w) == (rank, world)
        dev = torch.device("cpu")
        names = [f"t{i}" for i in range(8)]
        sizes = [64, 8, 32, 16, 16, 3, 1, 0]   # odd byte counts: 16-B aligned slots; an empty tensor
        owner = dict(zip(names, D.shard(sizes, world)))
        shapes = {n: {"qweight": ((s, 2), torch.int32), "scales": ((s,), torch.float16)} for n, s in zip(names, sizes)}
        def content(i, s):     # random bits, NaN / inf patterns included (byte-exact transfer)
            g = torch.Generator().manual_seed(i)
            qw = torch.randint(-2 ** 31, 2 ** 31 - 1, (s, 2), generator=g, dtype=torch.int64).to(torch.int32)
            sc = torch.randint(-2 ** 15, 2 ** 15 - 1, (s,), generator=g, dtype=torch.int32).to(torch.int16)
            return qw, sc.view(torch.float16)
        local = {}
        for i, (n, s) in enumerate(zip(names, sizes)):
            if owner[n] == rank:
                qw, sc = content(i, s)
                local[n] = {"qweight": qw, "scales": sc}
        merged = D.gather_to_rank0(local, owner, shapes, dev)
        t = D.max_over_ranks(float(rank + 1), dev)
        fl = D.all_gather_floats([float(rank), 2.5 * rank], dev)
        D.barrier()
        if rank == 0:
            ok = sorted(merged) == sorted(names) and t == float(world)
            ok &= fl == [[float(r), 2.5 * r] for r in range(world)]
            # one receive buffer per (peer, field): the merged fields are views carved from it,
            # disjoint, and together exactly the peers' result bytes (no staging, no clone)
            spans, total = [], 0
            for i, (n, s) in enumerate(zip(names, sizes)):
                qw, sc = content(i, s)
                ok &= bool(torch.equal(merged[n]["qweight"], qw))
                ok &= bool(torch.equal(merged[n]["scales"].view(torch.int16), sc.view(torch.int16)))
                for f, v in merged[n].items():
                    if owner[n] != 0 and v.numel():
                        b = v.data_ptr()
                        spans.append((b, b + v.numel() * v.element_size()))
                        total += v.numel() * v.element_size()
            spans.sort()
            ok &= all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
            bufs = {v.untyped_storage().data_ptr(): v.untyped_storage().nbytes()
                    for n in names if owner[n] != 0 for v in merged[n].values() if v.numel()}
            ok &= sum(bufs.values()) == total
            ok &= len(bufs) <= 2 * (world - 1)
            import io
            torch.save(merged, io.BytesIO())   # results own their storage (the CLI saves them)
            q.put(("ok" if ok else "mismatch", sorted(merged)))
        dist.destroy_process_group()
    except Exception as e:  # surface to the parent
        q.put(("error", repr(e)))
        raise


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_and_timing(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=150)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == "ok", res
    assert all(p.exitcode == 0 for p in procs)


def _llama70b_names_shapes():
    """The Llama-3-70B tensor set (723 tensors) with its real names."""
    h, inter, kv, vocab = 8192, 28672, 1024, 128256
    t = {"model.embed_tokens.weight": (vocab, h), "lm_head.weight": (vocab, h), "model.norm.weight": (h,)}
    for l in range(80):
        p = f"model.layers.{l}."
        t.update({p + "self_attn.q_proj.weight": (h, h), p + "self_attn.k_proj.weight": (kv, h),
                  p + "self_attn.v_proj.weight": (kv, h), p + "self_attn.o_proj.weight": (h, h),
                  p + "mlp.gate_proj.weight": (inter, h), p + "mlp.up_proj.weight": (inter, h),
                  p + "mlp.down_proj.weight": (h, inter), p + "input_layernorm.weight": (h,),
                  p + "post_attention_layernorm.weight": (h,)})
    return t


def _scaled_packed(i, shape, div=256):
    """Packed-format result fields of tensor i with its rows scaled down by `div` (K kept):
    random bits, so a misplaced or truncated byte shows."""
    rows = max(1, shape[0] // div) if len(shape) > 1 else 1
    K = shape[-1]
    G = -(-K // 128)
    g = torch.Generator().manual_seed(1000 + i)
    return {"qweight": torch.randint(-2 ** 31, 2 ** 31 - 1, (rows, -(-K // 8)), generator=g, dtype=torch.int64).to(torch.int32),
            "qzeros": torch.randint(-2 ** 31, 2 ** 31 - 1, (rows, -(-G // 8)), generator=g, dtype=torch.int64).to(torch.int32),
            "scales": torch.randint(-2 ** 15, 2 ** 15 - 1, (rows, G), generator=g, dtype=torch.int32).to(torch.int16).view(torch.float16)}


def _worker70b(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        D.init("gloo")
        dev = torch.device("cpu")
        ts = _llama70b_names_shapes()
        names = list(ts)
        nbytes = [2 * int(torch.Size(ts[n]).numel()) for n in names]
        owner = dict(zip(names, D.shard(nbytes, world)))      # the real shapes' LPT map
        shapes = {}
        for i, n in enumerate(names):
            r = _scaled_packed(i, ts[n]) if owner[n] == rank or rank == 0 else None
            if r is None:       # shapes alone (every rank derives them from the header index)
                rows = max(1, ts[n][0] // 256) if len(ts[n]) > 1 else 1
                K = ts[n][-1]
                G = -(-K // 128)
                shapes[n] = {"qweight": ((rows, -(-K // 8)), torch.int32), "qzeros": ((rows, -(-G // 8)), torch.int32),
                             "scales": ((rows, G), torch.float16)}
            else:
                shapes[n] = {f: (tuple(v.shape), v.dtype) for f, v in r.items()}
        # this rank's results as views of ONE arena per field (the native pipeline's layout):
        # they go out without a copy
        mine = [n for n in sorted(owner) if owner[n] == rank]
        local = {}
        for f in ("qweight", "qzeros", "scales"):
            parts = [_scaled_packed(names.index(n), ts[n])[f] for n in mine]
            if not parts:
                continue
            arena = torch.cat([p.reshape(-1) for p in parts])
            off = 0
            for n, p in zip(mine, parts):
                local.setdefault(n, {})[f] = arena[off:off + p.numel()].view(p.shape)
                off += p.numel()
            if rank:
                assert D._flat_view([local[n][f] for n in mine]) is not None
        plan = D.gather_plan(owner, shapes, world)
        merged = D.gather_to_rank0(local, owner, shapes, dev)
        D.barrier()
        if rank == 0:
            ok = len(plan) == 3 * (world - 1) and sorted(merged) == sorted(names)
            for i, n in enumerate(names):
                want = _scaled_packed(i, ts[n])
                for f, v in want.items():
                    ok &= bool(torch.equal(merged[n][f].view(torch.int16) if f == "scales" else merged[n][f],
                                           v.view(torch.int16) if f == "scales" else v))
            q.put(("ok" if ok else "mismatch", len(plan)))
        dist.destroy_process_group()
    except Exception as e:  # surface to the parent
        q.put(("error", repr(e)))
        raise


@pytest.mark.timeout(240)
def test_gloo_world8_llama70b_gather():
    """world 8 on the Llama-3-70B ownership map (723 names, LPT over the
    real byte sizes, rows scaled down 256x), byte-exact at rank 0, 21 point-to-point
    messages (7 peers x 3 fields) instead of one per tensor and field."""
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker70b, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=200)
    for p in procs:
        p.join(timeout=60)
    assert res == ("ok", 21), res
    assert all(p.exitcode == 0 for p in procs)
