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
            ptrs = set()
            for i, (n, s) in enumerate(zip(names, sizes)):
                qw, sc = content(i, s)
                ok &= bool(torch.equal(merged[n]["qweight"], qw))
                ok &= bool(torch.equal(merged[n]["scales"].view(torch.int16), sc.view(torch.int16)))
                for f, v in merged[n].items():
                    # bounded receive footprint: every received field is its own exact-size
                    # allocation (no staging buffer behind views, no second copy)
                    if owner[n] != 0 and v.numel():
                        ok &= v.untyped_storage().nbytes() == v.numel() * v.element_size()
                        ok &= v.data_ptr() not in ptrs
                        ptrs.add(v.data_ptr())
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
