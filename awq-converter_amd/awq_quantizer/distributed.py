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
    straight from the senders' result tensors into rank 0's final output tensors (batched
    isend/irecv: over xGMI each peer has its own link to rank 0, so the 7 senders do not
    share bandwidth; a ring/all-gather would move 7x the bytes).

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


def gather_to_rank0(local: Dict[str, Dict[str, torch.Tensor]], owner: Dict[str, int],
                    shapes: Dict[str, Dict[str, Tuple[Tuple[int, ...], torch.dtype]]],
                    device: torch.device) -> Dict[str, Dict[str, torch.Tensor]]:
    """Send every rank's results to rank 0.

    local:  this rank's results, name -> {field: tensor on `device`}
    owner:  name -> owning rank (from shard(); identical everywhere)
    shapes: name -> {field: (shape, dtype)} of every result (derivable from the header
            index, identical everywhere) so rank 0 can post its receives up front.
    Returns the merged dict on rank 0 and `local` elsewhere.

    Zero-copy on both ends: rank 0 allocates each result field once, at its final shape and
    dtype, and receives straight into it; a sender sends its own result tensors as they are.
    Rank 0's receive footprint is therefore exactly the merged outputs (no staging buffers,
    no clones).  All transfers go out as one batch of point-to-point operations, so each
    peer streams over its own xGMI link into rank 0 concurrently with the others.
    """
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return local
    rank, world = dist.get_rank(), dist.get_world_size()
    ops, merged = [], {}
    for name in sorted(owner):          # the same order on every rank: sends and receives pair up
        src = owner[name]
        if src == 0 or rank not in (0, src):
            continue
        for field in sorted(shapes[name]):
            shp, dt = shapes[name][field]
            if torch.Size(shp).numel() == 0:
                continue
            if rank == 0:
                t = torch.empty(shp, dtype=dt, device=device)
                merged.setdefault(name, {})[field] = t
                ops.append(dist.P2POp(dist.irecv, t, src))
            else:
                ops.append(dist.P2POp(dist.isend, local[name][field].contiguous(), 0))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != 0:
        return local
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
