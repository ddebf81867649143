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
    one coalesced message per peer (batched isend/irecv: over xGMI each peer has its own
    link to rank 0, so the 7 senders do not share bandwidth; a ring/all-gather would move
    7x the bytes).

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


def _layout(names: Sequence[str], shapes: Dict[str, Dict[str, Tuple[Tuple[int, ...], torch.dtype]]]):
    """Byte offsets of every (name, field) in one peer's flat message, 16-B aligned so every
    slice can be viewed back as its dtype; identical on sender and receiver."""
    off, lay = 0, []
    for name in names:
        for field in sorted(shapes[name]):
            shp, dt = shapes[name][field]
            nb = int(torch.Size(shp).numel()) * torch.empty((), dtype=dt).element_size()
            lay.append((name, field, off, nb, tuple(shp), dt))
            off += -(-nb // 16) * 16
    return lay, off


def gather_to_rank0(local: Dict[str, Dict[str, torch.Tensor]], owner: Dict[str, int],
                    shapes: Dict[str, Dict[str, Tuple[Tuple[int, ...], torch.dtype]]],
                    device: torch.device) -> Dict[str, Dict[str, torch.Tensor]]:
    """Send every rank's results to rank 0.

    local:  this rank's results, name -> {field: tensor on `device`}
    owner:  name -> owning rank (from shard(); identical everywhere)
    shapes: name -> {field: (shape, dtype)} of every result (derivable from the header
            index, identical everywhere) so rank 0 can post its receives up front.
    Returns the merged dict on rank 0 and `local` elsewhere.

    One message per peer: each sender coalesces its results into one flat byte buffer
    (a device copy of ~0.52 B per quantized element, in the layout _layout() derives from
    `shapes`), so the exchange is world-1 large point-to-point transfers in one batch —
    each over its own xGMI link into rank 0 — instead of one small message per tensor field.
    """
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return local
    rank, world = dist.get_rank(), dist.get_world_size()
    by_rank: Dict[int, List[str]] = {}
    for name in sorted(owner):
        by_rank.setdefault(owner[name], []).append(name)
    ops, recv = [], {}
    for src in range(1, world):
        lay, total = _layout(by_rank.get(src, []), shapes)
        if total == 0:
            continue
        if rank == 0:
            buf = torch.empty(total, dtype=torch.uint8, device=device)
            recv[src] = (buf, lay)
            ops.append(dist.P2POp(dist.irecv, buf, src))
        elif rank == src:
            buf = torch.empty(total, dtype=torch.uint8, device=device)
            for name, field, off, nb, _, _ in lay:
                t = local[name][field].contiguous()
                if nb:
                    buf[off:off + nb].copy_(t.reshape(-1).view(torch.uint8))
            ops.append(dist.P2POp(dist.isend, buf, 0))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != 0:
        return local
    merged: Dict[str, Dict[str, torch.Tensor]] = {n: local[n] for n in by_rank.get(0, [])}
    for src in list(recv):
        buf, lay = recv.pop(src)
        # own storage per result (a device copy): views of one buffer under different dtypes
        # cannot be torch.save'd, and the receive buffer is freed peer by peer
        for name, field, off, nb, shp, dt in lay:
            merged.setdefault(name, {})[field] = buf[off:off + nb].view(dt).view(shp).clone()
        del buf
    return {n: merged[n] for n in owner}
