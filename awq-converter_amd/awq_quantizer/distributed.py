"""Multi-GPU plumbing: one process per GPU (torchrun), torch.distributed (RCCL on ROCm).

Weights quantize independently, tensor by tensor, so the data path needs NO collective:
every rank quantizes its own share and there is no exchange during the hot loop.  The
only communication is optional and happens after it:

  * shard(): LPT partition of a tensor list by bytes (the reference's own
    partition_tensors, src/awq_quantizer/main.py:395-427, which it never calls) —
    deterministic, so every rank derives the same ownership map from the same header
    index without exchanging anything;
  * max_over_ranks(): the bench's max-of-ranks wall time;
  * gather_to_rank0(): point-to-point transfer of every rank's packed outputs to rank 0,
    one flat message per peer and field, received into buffers rank 0's results are views
    of (batched isend/irecv: over xGMI each peer has its own link to rank 0, so the 7
    senders do not share bandwidth; a ring/all-gather would move 7x the bytes).

Everything here runs with the gloo backend on CPU as well (tests/test_distributed.py).
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import torch
import torch.distributed as dist


def env_world() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (1 process: 0, 0, 1)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend: str = "nccl") -> Tuple[int, int, int]:
    """Initialise the default process group if WORLD_SIZE > 1; returns (rank, local, world)."""
    rank, local, world = env_world()
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, local, world


def shard(sizes: Sequence[int], world: int) -> List[int]:
    """Owner rank of every item: greedy LPT by size (largest first, ties by index, to the
    least-loaded rank, lowest rank on ties).  Deterministic and identical on every rank."""
    order = sorted(range(len(sizes)), key=lambda i: (-int(sizes[i]), i))
    load = [0] * max(1, world)
    owner = [0] * len(sizes)
    for i in order:
        r = min(range(len(load)), key=lambda k: (load[k], k))
        owner[i] = r
        load[r] += int(sizes[i])
    return owner


def barrier() -> None:
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def max_over_ranks(value: float, device: torch.device) -> float:
    """Max of a per-rank float over all ranks (the bench's wall time)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(value)
    if dist.get_backend() != "nccl":
        device = torch.device("cpu")
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_floats(values: Sequence[float], device: torch.device) -> List[List[float]]:
    """Every rank's small list of floats (same length everywhere), rank-ordered."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return [list(map(float, values))]
    if dist.get_backend() != "nccl":
        device = torch.device("cpu")
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def _flat_view(ts: List[torch.Tensor]):
    """A 1-D view covering `ts` when they already lie back to back, in order, in one storage
    (e.g. results carved from one arena); None otherwise."""
    first = ts[0]
    st = first.untyped_storage()
    es = first.element_size()
    off = first.storage_offset()
    for t in ts:
        if (t.dtype != first.dtype or not t.is_contiguous() or t.untyped_storage().data_ptr() != st.data_ptr()
                or t.storage_offset() != off):
            return None
        off += t.numel()
    if off * es > st.nbytes():
        return None
    return torch.empty(0, dtype=first.dtype, device=first.device).set_(st, first.storage_offset(),
                                                                        (off - first.storage_offset(),))


def gather_plan(owner: Dict[str, int], shapes: Dict[str, Dict[str, Tuple[Tuple[int, ...], torch.dtype]]],
                world: int):
    """The transfers of gather_to_rank0, identical on every rank: for every peer p >= 1 and
    every (field, dtype), the peer's names (sorted) holding that field and their element
    counts — one flat message each, so a world of W ranks moves at most (W - 1) x fields
    point-to-point messages whatever the number of tensors."""
    plan = []
    names = sorted(owner)
    for p in range(1, world):
        mine = [n for n in names if owner[n] == p]
        keys = sorted({(f, str(dt)) for n in mine for f, (_, dt) in shapes[n].items()})
        for f, dts in keys:
            items = [(n, tuple(shapes[n][f][0])) for n in mine
                     if f in shapes[n] and str(shapes[n][f][1]) == dts]
            counts = [int(torch.Size(shp).numel()) for _, shp in items]
            if sum(counts):
                plan.append((p, f, shapes[items[0][0]][f][1], items, counts))
    return plan


def gather_to_rank0(local: Dict[str, Dict[str, torch.Tensor]], owner: Dict[str, int],
                    shapes: Dict[str, Dict[str, Tuple[Tuple[int, ...], torch.dtype]]],
                    device: torch.device) -> Dict[str, Dict[str, torch.Tensor]]:
    """Send every rank's results to rank 0.

    local:  this rank's results, name -> {field: tensor on `device`}
    owner:  name -> owning rank (from shard(); identical everywhere)
    shapes: name -> {field: (shape, dtype)} of every result (derivable from the header
            index, identical everywhere) so rank 0 can post its receives up front.
    Returns the merged dict on rank 0 and `local` elsewhere.

    One message per peer and field (gather_plan): a peer sends all its tensors' values of
    one field as one flat buffer (its results themselves when they already lie back to back
    in one arena, else one device-side concatenation), rank 0 receives it into one flat
    buffer and its result fields are views carved from it — no clone, and rank 0's receive
    footprint is exactly the merged outputs.  At world 8 on the Llama-3-70B set that is 21
    messages instead of one per tensor and field (~1 900), all posted as one batch, so each
    peer streams over its own xGMI link into rank 0 concurrently with the others.
    """
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return local
    rank, world = dist.get_rank(), dist.get_world_size()
    ops, recv = [], []
    for p, f, dt, items, counts in gather_plan(owner, shapes, world):
        if rank == 0:
            flat = torch.empty(sum(counts), dtype=dt, device=device)
            recv.append((flat, f, items, counts))
            ops.append(dist.P2POp(dist.irecv, flat, p))
        elif rank == p:
            ts = [local[n][f] for n, _ in items]
            flat = _flat_view(ts)
            if flat is None:
                flat = torch.cat([t.reshape(-1) for t in ts])
            ops.append(dist.P2POp(dist.isend, flat, 0))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != 0:
        return local
    merged: Dict[str, Dict[str, torch.Tensor]] = {}
    for flat, f, items, counts in recv:
        off = 0
        for (n, shp), c in zip(items, counts):
            merged.setdefault(n, {})[f] = flat[off:off + c].view(shp)
            off += c
    for name in owner:
        if owner[name] == 0:
            merged[name] = local[name]
        else:       # (empty fields of a peer's result: nothing crossed the fabric)
            d = merged.setdefault(name, {})
            for field in shapes[name]:
                if field not in d:
                    shp, dt = shapes[name][field]
                    d[field] = torch.empty(shp, dtype=dt, device=device)
    return {n: merged[n] for n in owner}
