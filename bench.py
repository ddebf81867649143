#!/usr/bin/env python3
"""Throughput bench of the AWQ group-quantize hot path on MI355X.

Metric (BASELINE.json): bf16 GB quantized/sec at group_size=128 (input bytes, 2 B/elem),
plus the HBM-roofline fraction of the quantize+pack kernel.

A *step* = one ragged launch of the streaming kernel over a whole synthetic tensor set
with the exact shapes of the named model, bits=4, group_size=128,
asymmetric (the CLI default, reference main.py:59-63), outputs = packed qweight/qzeros +
fp16 scales, inputs resident in HBM.  Multi-GPU: one process per GPU (torchrun); every
rank quantizes its own replica of the tensor set (weak scaling, no data-path collective:
tensors are independent).  value = all ranks' input bytes / max-over-ranks time.
--shard: strong scaling instead — one copy of the set, its tensor list LPT-sharded over the
ranks (the CLI's torchrun mode), value = the set's bytes / max-over-ranks time.

Usage: python bench.py [--gpus N --steps K --warmup W --workload opt-125m]
       N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "awq-converter_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

METRIC = "bf16 GB quantized/sec at group_size=128, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md); 6.29 TB/s measured copy

# Shape manifests (every float tensor with numel >= 128 = the
# reference CLI's filter, main.py:244-253).
WORKLOADS = {
    "c1": [((1024, 4096), 1)],
    "opt-125m": [((768,), 110), ((768, 768), 48), ((3072, 768), 12), ((3072,), 12), ((768, 3072), 12),
                 ((50272, 768), 1), ((2050, 768), 1)],
    "opt-350m": [((1024,), 216), ((1024, 1024), 96), ((4096, 1024), 24), ((4096,), 24), ((1024, 4096), 24),
                 ((50272, 512), 1), ((2050, 1024), 1), ((512, 1024), 1), ((1024, 512), 1)],
    "llama3-8b": [((4096,), 65), ((4096, 4096), 64), ((1024, 4096), 64), ((14336, 4096), 64),
                  ((4096, 14336), 32), ((128256, 4096), 2)],
    "llama3-70b": [((8192,), 161), ((8192, 8192), 160), ((1024, 8192), 160), ((28672, 8192), 160),
                   ((8192, 28672), 80), ((128256, 8192), 2)],
}
DESCR = {"c1": "single 1024x4096 linear", "opt-125m": "facebook/opt-125m tensor set (196 tensors, 125.24M params)",
         "opt-350m": "facebook/opt-350m tensor set (388 tensors, 331.2M params)",
         "llama3-8b": "Llama-3-8B tensor set (291 tensors, 8.03B params)",
         "llama3-70b": "Llama-3-70B tensor set (723 tensors, 70.55B params)"}


def shapes_of(workload):
    out = []
    for shape, count in WORKLOADS[workload]:
        out += [shape] * count
    # processing order of the reference CLI: bytes descending, stable (main.py:259)
    return sorted(out, key=lambda s: -int(torch.Size(s).numel()))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # Defaults measure the sustained rate: the chip's clocks settle only after ~20-30 ms of
    # back-to-back launches (scripts/sustain_probe.py, profiles/r60: opt-125m launches run
    # 54-66 us during the first ~300, then a steady 53.9 us), so 500 warmup launches
    # (~28 ms) precede 1000 timed ones (~54 ms; the ~35 us launch / sync edge of the timed
    # region is then < 0.1 %).
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--workload", default="opt-125m", choices=sorted(WORKLOADS))
    ap.add_argument("--bits", type=int, default=4, choices=[4, 8])
    ap.add_argument("--symmetric", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "f32"],
                    help="bf16 = the BASELINE metric; f16 / f32 are extra lines (metric names the dtype)")
    ap.add_argument("--group-size", type=int, default=128, choices=[32, 64, 128, 256],
                    help="128 = the BASELINE metric; other sizes are extra lines (metric names the size)")
    ap.add_argument("--parity", action="store_true", help="also write unpacked int32 tensor_q/zero_points")
    ap.add_argument("--shard", action="store_true",
                    help="strong scaling: ONE copy of the tensor set, its tensor list LPT-sharded across the "
                         "ranks (distributed.shard, the CLI's torchrun mode; SURVEY 8e) instead of a replica "
                         "per rank")
    ap.add_argument("--replicas", type=int, default=0,
                    help="input replicas rotated across steps (0 = enough to exceed the 256 MiB Infinity Cache)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-seconds", type=float, default=15.0)
    ap.add_argument("--events", default="span", choices=["step", "span"])
    ap.add_argument("--no-copy-ceiling", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the (untimed) gather-to-rank-0 leg")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


DTYPES = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}


def make_set(shapes, seed0, dev, dtype=torch.bfloat16, only=None):
    """Synthetic N(0, 0.02) tensors, tensor i seeded by seed0 + i; `only`: the indices to
    materialise (a rank's shard)."""
    g = torch.Generator(device=dev)
    tensors = {}
    for i, s in enumerate(shapes):
        if only is not None and i not in only:
            continue
        g.manual_seed(seed0 + i)
        tensors[f"t{i:04d}"] = (torch.randn(*s, generator=g, device=dev, dtype=torch.float32) * 0.02).to(dtype)
    return tensors


def copy_ceiling(dev, stream, nbytes=1 << 30, iters=10):
    """HBM copy of `nbytes` (read + write counted) by the library's stream-copy kernel, which
    has the quantizer's memory structure (one wave per 4 KiB, 16-B nt accesses): the
    achievable-bandwidth reference SURVEY.md §8(d) asks the kernel to be quoted against."""
    from awq_quantizer import _hip
    src = torch.empty(nbytes // 4, dtype=torch.int32, device=dev).fill_(1)
    dst = torch.empty_like(src)
    for _ in range(3):
        _hip.stream_copy(src, dst, stream.cuda_stream)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(iters):
        _hip.stream_copy(src, dst, stream.cuda_stream)
    b.record(stream)
    torch.cuda.synchronize()
    gbs = 2 * nbytes * iters / (a.elapsed_time(b) / 1e3) / 1e9
    del src, dst
    return gbs


def cpu_threads():
    """Host threads for the CPU baseline: OMP_NUM_THREADS if set (16 on the GPU box),
    else the CPUs this process may run on."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_baseline(shapes, budget_s, group_size=128, dtype=torch.bfloat16):
    """The oracle (oracle/awq_oracle.c, OpenMP over rows) on a bounded sample of the SAME
    workload: the tensor set in processing order, pass after pass, until about budget_s of
    CPU work (the last tensor may be cut to a row block).  Returns (GB/s of input,
    seconds, bytes, tensors, threads)."""
    from oracle import awq_oracle as orc
    threads = orc.set_threads(cpu_threads())
    g = torch.Generator().manual_seed(1234)
    done_bytes, t_total, parts = 0, 0.0, 0
    cache = {}
    while t_total < budget_s - 0.2:
        for s in shapes:
            rows = 1 if len(s) == 1 else s[0]
            K = int(torch.Size(s).numel()) // rows
            remaining = budget_s - t_total
            if remaining <= 0.2:
                break
            take = rows
            est = 3e-8 * rows * K / threads
            if est > remaining:
                take = max(1, int(rows * remaining / est))
            key = (take, K)
            if key not in cache:
                cache[key] = (torch.randn(take, K, generator=g) * 0.02).to(dtype)
            x = cache[key]
            t0 = time.perf_counter()
            orc.quantize_groups(x, take, K, group_size, 4, False)
            t_total += time.perf_counter() - t0
            done_bytes += x.numel() * x.element_size()
            parts += 1
    return done_bytes / t_total / 1e9, t_total, done_bytes, parts, threads


def packed_out_shapes(shape, bits, gs):
    """qweight / qzeros / scales shapes and dtypes of one tensor's packed outputs (PackedBatch)."""
    rows = 1 if len(shape) <= 1 else shape[0]
    K = int(torch.Size(shape).numel()) // rows
    G, per = -(-K // gs), 32 // bits
    return {"qweight": ((rows, -(-K // per)), torch.int32), "qzeros": ((rows, -(-G // per)), torch.int32),
            "scales": ((rows, G), torch.float16)}


def gather_leg(batch, rank, world, dev, backend, iters=3, shard_owner=None, all_shapes=None, bits=4, gs=128):
    """N>1 only, after the timed region: the CLI's exchange step (distributed.gather_to_rank0,
    one coalesced message per peer) on every rank's packed outputs of one replica (or, with
    --shard, of its shard: the real exchange of the CLI's torchrun mode).  Reported beside
    `value`, never inside it (the gather is a separate line)."""
    from awq_quantizer import distributed as D
    comm = dev if backend == "nccl" else torch.device("cpu")
    fields = ("qweight", "qzeros", "scales")
    owner, shapes = {}, {}
    if shard_owner is None:
        for r in range(world):
            for n in batch.names:
                owner[f"{r}/{n}"] = r
                shapes[f"{r}/{n}"] = {f: (tuple(batch.out[n][f].shape), batch.out[n][f].dtype) for f in fields}
        local = {f"{rank}/{n}": {f: batch.out[n][f].to(comm) for f in fields} for n in batch.names}
    else:
        for i, r in enumerate(shard_owner):
            owner[f"t{i:04d}"] = r
            shapes[f"t{i:04d}"] = packed_out_shapes(all_shapes[i], bits, gs)
        local = {n: {f: batch.out[n][f].to(comm) for f in fields} for n in batch.names}
    per_rank = sum(batch.out[n][f].numel() * batch.out[n][f].element_size() for n in batch.names for f in fields)
    D.gather_to_rank0(local, owner, shapes, comm)                     # warmup (connects the P2P channels)
    torch.cuda.synchronize(dev)
    D.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        D.gather_to_rank0(local, owner, shapes, comm)
    torch.cuda.synchronize(dev)
    D.barrier()
    t = D.max_over_ranks((time.perf_counter() - t0) / iters, dev)
    if shard_owner is None:
        moved = per_rank * (world - 1)
    else:
        moved = sum(int(torch.Size(sh).numel()) * torch.empty((), dtype=dt).element_size()
                    for i, r in enumerate(shard_owner) if r != 0 for sh, dt in shapes[f"t{i:04d}"].values())
    what = ("gather of the other ranks' packed shards to rank 0" if shard_owner is not None else
            "gather of every rank's packed outputs (one replica) to rank 0")
    return {"what": what + f", one P2P message per peer ({backend}); outside the timed region",
            "bytes_to_rank0": moved, "ms": round(t * 1e3, 3), "GBs_into_rank0": round(moved / t / 1e9, 2)}


def main():
    args = parse()
    from awq_quantizer import _hip
    from awq_quantizer import distributed as D
    from awq_quantizer.quantization.batch import PackedBatch
    # RCCL, one process per GPU (torchrun).  AWQ_DIST_BACKEND=gloo only to rehearse the
    # N>1 path with several ranks on one GPU (RCCL refuses two ranks on one device).
    backend = os.environ.get("AWQ_DIST_BACKEND", "nccl")
    rank, local, world = D.init(backend)
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    _hip.require_device(dev)

    all_shapes = shapes_of(args.workload)
    dtype = DTYPES[args.dtype]
    esize = torch.empty((), dtype=dtype).element_size()
    if args.shard:
        # strong scaling: rank r quantizes the tensors LPT assigns it (tensor i is seeded by
        # its index, so the data do not depend on the world size)
        owner = D.shard([int(torch.Size(s).numel()) for s in all_shapes], world)
        mine = [i for i in range(len(all_shapes)) if owner[i] == rank]
    else:
        mine = list(range(len(all_shapes)))
    shapes = [all_shapes[i] for i in mine]
    elems = sum(int(torch.Size(s).numel()) for s in shapes)
    total_elems = sum(int(torch.Size(s).numel()) for s in all_shapes)
    in_bytes = elems * esize
    # bytes all ranks quantize per step: the whole set once (shard) or one replica per rank
    step_bytes = total_elems * esize if args.shard else in_bytes * world
    reps = args.replicas or max(1, -(-(1 << 30) // max(1, in_bytes)))   # >= 1 GiB of inputs in rotation
    batches = []
    for r in range(reps):
        if args.shard:
            inputs = make_set(all_shapes, r * 100003, dev, dtype, only=set(mine))
        else:
            inputs = make_set(shapes, (rank * 64 + r) * 100003, dev, dtype)
        batches.append(PackedBatch(inputs, bits=args.bits, symmetric=args.symmetric, parity=args.parity,
                                   group_size=args.group_size))
    torch.cuda.synchronize()
    algo_bytes = batches[0].algorithmic_bytes()

    barrier = D.barrier
    stream = torch.cuda.current_stream(dev)
    for i in range(args.warmup):
        batches[i % reps].run(stream)
    torch.cuda.synchronize()

    # HIP events on the kernel's stream.  "span" (default): one pair around the K back-to-back
    # launches -> average launch duration incl. the sub-us dispatch gaps; it agrees with the
    # rocprofv3 kernel average within ~1.5 % (profiles/r15_*).  "step": a pair around every
    # launch; each marker adds ~4 us to the queue (r15: 70.5 us vs rocprof 67.8 us).
    n_ev = args.steps if args.events == "step" else 1
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_ev)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.events == "step":
        for i in range(args.steps):
            ev[i][0].record(stream)
            batches[i % reps].run(stream)
            ev[i][1].record(stream)
    else:
        ev[0][0].record(stream)
        for i in range(args.steps):
            batches[i % reps].run(stream)
        ev[0][1].record(stream)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    kern_avg_s = sum(kern_ms) / args.steps / 1e3
    ceiling = None if args.no_copy_ceiling or rank != 0 else copy_ceiling(dev, stream)

    elapsed = D.max_over_ranks(elapsed, dev)
    gather = (gather_leg(batches[0], rank, world, dev, backend, shard_owner=owner if args.shard else None,
                         all_shapes=all_shapes, bits=args.bits, gs=args.group_size)
              if world > 1 and not args.no_gather else None)

    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    value = step_bytes * args.steps / elapsed / 1e9
    achieved = algo_bytes / kern_avg_s / 1e9
    traffic = None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        key = f"{args.workload}.b{args.bits}.{'sym' if args.symmetric else 'asym'}.{'parity' if args.parity else 'packed'}"
        if args.group_size != 128:
            key += f".gs{args.group_size}"
        if args.dtype != "bf16":
            key += f".{args.dtype}"
        traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    line = {
        "metric": METRIC.replace("group_size=128", f"group_size={args.group_size}").replace("bf16", args.dtype),
        "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong" if args.shard else "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
        "config": {"workload": f"{args.workload}: {DESCR[args.workload]}", "tensors": len(all_shapes),
                   "elements": total_elems, "group_size": args.group_size, "bits": args.bits, "symmetric": args.symmetric,
                   "outputs": "qweight+qzeros+fp16 scales" + (" + int32 tensor_q/zero_points" if args.parity else ""),
                   "launches_per_step": 1, "input_replicas_rotated": reps,
                   "parallelism": (f"shard{world} (tensor list LPT-sharded over the ranks; rank 0 holds "
                                   f"{len(shapes)} tensors, {elems} elements)") if args.shard else
                                  f"dp{world} (each rank quantizes its own replica of the tensor set)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "kernel_avg_us": round(kern_avg_s * 1e6, 2), "timing": f"hip events ({args.events})"},
    }
    if gather:
        line["exchange"] = gather
    if ceiling:
        line["roofline"]["copy_ceiling"] = round(ceiling, 1)
        line["roofline"]["frac_of_copy"] = round(achieved / ceiling, 4)
    if not args.no_cpu_baseline:
        gbs, secs, nbytes, nparts, threads = cpu_baseline(shapes, args.cpu_sample_seconds, args.group_size, dtype)
        line["cpu_baseline"] = {"value": round(gbs, 5), "unit": "GB/s", "cores": threads, "kind": "port",
                                "sample": f"oracle/awq_oracle.c (OpenMP over rows, {threads} threads) on "
                                          f"{nbytes / 1e6:.1f} MB of the {args.workload} set ({nparts} tensors/row-"
                                          f"blocks in processing order, repeated passes, {secs:.1f} s); reference "
                                          f"awq.py itself: 4.6 MB/s on 1 core, 23.6 MB/s on 8 (BASELINE.md)"}
    print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
