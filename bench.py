#!/usr/bin/env python3
"""Throughput bench of the AWQ group-quantize hot path on MI355X.

Metric (BASELINE.json): bf16 GB quantized/sec at group_size=128 (input bytes, 2 B/elem),
plus the HBM-roofline fraction of the quantize+pack kernel.

Default workload = the north_star set: the Llama-3-70B tensor list (723 tensors, 70.55 G
elements, 141 GB bf16), which fits one MI355X (141 GB in + 37 GB
packed out of 288 GB).  A *step* = one ragged launch of the streaming kernel over the
rank's tensors, bits=4, group_size=128, asymmetric (the CLI default, reference
main.py:59-63), outputs = packed qweight/qzeros + fp16 scales, inputs resident in HBM.

Multi-GPU (default): one process per GPU (torchrun), ONE copy of the tensor set, its
tensor list LPT-sharded over the ranks exactly as the CLI's torchrun mode does (the
reference's own partition_tensors, main.py:395-427) -> "scaling": "strong", value = the
set's bytes / max-over-ranks time.  The exchange (gather of the packed shards to rank 0,
RCCL point-to-point over xGMI) runs after the timed region and is reported as "exchange".
--replica: weak scaling instead (every rank quantizes its own copy of the set).

Clocks: the chip's clocks settle only after ~20-30 ms of back-to-back HBM streaming
(profiles/r60_sustain_probe.log), so the read-dominant ceiling probe (>= 150 ms of
streaming) runs on every rank BEFORE the warmup launches, whatever --warmup is.

Usage: python bench.py [--gpus N --steps K --warmup W --workload llama3-70b]
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
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

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
# reference awq.py itself, measured in the survey container
REFERENCE_CPU = "reference awq.py itself: 4.61 MB/s on 1 process (8 torch threads), 23.6 MB/s with 8 processes (BASELINE.md)"


def shapes_of(workload):
    out = []
    for shape, count in WORKLOADS[workload]:
        out += [shape] * count
    # processing order of the reference CLI: bytes descending, stable (main.py:259)
    return sorted(out, key=lambda s: -int(torch.Size(s).numel()))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # Llama-3-70B: one launch is ~30 ms, so 20 timed launches are ~0.6 s of kernel time
    ap.add_argument("--steps", type=int, default=60)   # ~1.7 s timed on the 70B set: long enough for a sampling GPU-busy probe
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="llama3-70b", choices=sorted(WORKLOADS))
    ap.add_argument("--bits", type=int, default=4, choices=[4, 8])
    ap.add_argument("--symmetric", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "f32"],
                    help="bf16 = the BASELINE metric; f16 / f32 are extra lines (metric names the dtype)")
    ap.add_argument("--group-size", type=int, default=128, choices=[32, 64, 128, 256],
                    help="128 = the BASELINE metric; other sizes are extra lines (metric names the size)")
    ap.add_argument("--parity", action="store_true", help="also write unpacked int32 tensor_q/zero_points")
    ap.add_argument("--replica", action="store_true",
                    help="weak scaling: every rank quantizes its own replica of the tensor set, instead of the "
                         "default ONE copy LPT-sharded across the ranks (distributed.shard, the CLI's torchrun "
                         "mode; SURVEY 8e)")
    ap.add_argument("--shard", action="store_true", help="(the default; kept for old command lines)")
    ap.add_argument("--replicas", type=int, default=0,
                    help="input copies rotated across steps (0 = enough to exceed the 256 MiB Infinity Cache)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-seconds", type=float, default=15.0)
    ap.add_argument("--events", default="span", choices=["step", "span"])
    ap.add_argument("--no-copy-ceiling", action="store_true",
                    help="skip the read-dominant ceiling probe (it also warms the clocks before the warmup)")
    ap.add_argument("--clock-warm-ms", type=float, default=150.0,
                    help="ms of ceiling-probe streaming before the warmup launches (clock ramp)")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the (untimed) gather-to-rank-0 leg")
    ap.add_argument("--write-dir", default=None,
                    help="after the timed region: every rank copies its packed shard to the host and writes it as "
                         "chunk files into this directory (the CLI's per-rank output, main.ChunkWriter), reported as "
                         "\"write\" (max over ranks); the files are removed afterwards")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "round6", "pmc_traffic.json"))
    ap.add_argument("--mode", default="rtn", choices=["rtn", "search", "act"],
                    help="rtn = the BASELINE metric (round-to-nearest, the reference's arithmetic); search = the "
                         "opt-in per-group clip search (scale_method='search') in the same ragged launch; act = the "
                         "activation-aware search (scale_method='awq') of one Llama-3-8B block's layer groups. "
                         "search / act are VALU-bound: their roofline is the VALU issue rate (extra lines)")
    ap.add_argument("--search-grid", type=int, default=20)
    ap.add_argument("--search-candidates", type=int, default=10,
                    help="--mode search: candidates of the grid (AWQQuantizer default: 20 x 0.5 = 10)")
    ap.add_argument("--act-tokens", type=int, default=512, help="--mode act: calibration tokens per layer group")
    ap.add_argument("--valu-json", default=os.path.join(ROOT, "profiles", "round6", "pmc_valu.json"))
    a = ap.parse_args(argv)
    if a.mode == "search" and not 1 < a.search_candidates <= a.search_grid:
        ap.error("--search-candidates must be in (1, --search-grid]")
    if a.replica and a.shard:
        ap.error("--replica and --shard are exclusive")
    return a


DTYPES = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}


def make_set(shapes, seed0, dev, dtype=torch.bfloat16, only=None):
    """Synthetic N(0, 0.02) tensors, tensor i seeded by seed0 + i; `only`: the indices to
    materialise (a rank's shard).  Generated in row blocks so the fp32 temporary stays
    small next to a 141 GB set."""
    g = torch.Generator(device=dev)
    tensors = {}
    for i, s in enumerate(shapes):
        if only is not None and i not in only:
            continue
        g.manual_seed(seed0 + i)
        t = torch.empty(*s, device=dev, dtype=dtype)
        flat = t.view(s[0], -1) if len(s) > 1 else t.view(1, -1)
        step = max(1, (1 << 28) // flat.shape[1])
        for r0 in range(0, flat.shape[0], step):
            blk = flat[r0:r0 + step]
            blk.copy_(torch.randn(blk.shape, generator=g, device=dev, dtype=torch.float32).mul_(0.02))
        tensors[f"t{i:04d}"] = t
    return tensors


def stream_ceiling(dev, stream, warm_ms, nbytes=1 << 30, iters=20):
    """Read-dominant ceiling: the library's awq_stream_ceiling kernel (the quantizer's memory
    structure — one wave per 4 KiB, 16-B nt loads — and its read:write ratio, 4 : 1 against
    the packed quantizer's 4096 : 1064, without the arithmetic), read + write counted.  Runs
    first, for >= warm_ms of back-to-back streaming, so the timed region starts on settled
    clocks."""
    from awq_quantizer import _hip
    src = torch.empty(nbytes // 4, dtype=torch.int32, device=dev).fill_(1)
    dst = torch.empty(nbytes // 16, dtype=torch.int32, device=dev)
    t0 = time.perf_counter()
    while True:
        for _ in range(8):
            _hip.stream_ceiling(src, dst, stream.cuda_stream)
        torch.cuda.synchronize(dev)
        if (time.perf_counter() - t0) * 1e3 >= warm_ms:
            break
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(iters):
        _hip.stream_ceiling(src, dst, stream.cuda_stream)
    b.record(stream)
    torch.cuda.synchronize(dev)
    gbs = 1.25 * nbytes * iters / (a.elapsed_time(b) / 1e3) / 1e9
    del src, dst
    return gbs


def host_cpus():
    """(threads used, node CPUs, CPUs in this process's affinity set).  On the GPU box
    os.cpu_count() and the affinity set show the whole machine, while the box's CPU share
    is OMP_NUM_THREADS (16, set by the harness): the baseline uses that share."""
    node = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS", "")
    used = int(env) if env.isdigit() and int(env) > 0 else aff
    return min(used, aff), node, aff


def _time_oracle(x, rows, K, group_size, bits=4, search=None):
    from oracle import awq_oracle as orc
    t0 = time.perf_counter()
    orc.quantize_groups(x, rows, K, group_size, bits, False, search=search)
    return time.perf_counter() - t0


def cpu_baseline(workload, budget_s, group_size=128, dtype=torch.bfloat16, search=None):
    """The oracle (oracle/awq_oracle.c, OpenMP over rows, bit-exact restatement of awq.py)
    on the host cores, SURVEY §8(d): C1 (1024x4096, sigma 1) in full, then a row sample of
    every distinct shape of the workload, each extrapolated to the shape's full row count
    and multiplicity; value = the workload's input bytes / the extrapolated time."""
    from oracle import awq_oracle as orc
    threads, node, aff = host_cpus()
    orc.set_threads(threads)
    g = torch.Generator().manual_seed(1234)
    esize = torch.empty((), dtype=dtype).element_size()
    c1 = (torch.randn(1024, 4096, generator=torch.Generator().manual_seed(0))).to(dtype)
    _time_oracle(c1, 1024, 4096, group_size, search=search)              # warm (page-in, OpenMP pool)
    c1_s = min(_time_oracle(c1, 1024, 4096, group_size, search=search) for _ in range(3))
    per_shape = budget_s / len(WORKLOADS[workload])
    rate0 = 1024 * 4096 * esize / c1_s                                   # bytes/s, for sizing the samples
    total_s, sampled, lines = 0.0, 0, []
    for shape, count in WORKLOADS[workload]:
        rows = 1 if len(shape) == 1 else shape[0]
        K = int(torch.Size(shape).numel()) // rows
        # a sample of <= 128 MB (or the whole tensor), timed repeatedly for ~half the shape's share
        take = max(1, min(rows, int(per_shape * 0.5 * rate0 / (K * esize)), (128 << 20) // (K * esize)))
        x = (torch.randn(take, K, generator=g) * 0.02).to(dtype)
        t, reps = 0.0, 0
        while reps < 2 or (t < per_shape * 0.5 and reps < 1000):
            t += _time_oracle(x, take, K, group_size, search=search)
            reps += 1
        t_full = t / reps * rows / take
        total_s += t_full * count
        sampled += take * K * esize * reps
        lines.append(f"{shape}x{count}: {take}/{rows} rows")
    wl_bytes = sum(int(torch.Size(s).numel()) * c for s, c in WORKLOADS[workload]) * esize
    return {"value": round(wl_bytes / total_s / 1e9, 5), "unit": "GB/s", "cores": threads, "kind": "port",
            "node_cpus": node, "affinity_cpus": aff,
            "cores_note": (f"{threads} threads = the CPU share this GPU box grants one GPU (the pool sets "
                           f"OMP_NUM_THREADS={threads} and allots 16 CPUs per GPU; the {aff} CPUs of the affinity set "
                           f"belong to the whole 8-GPU node and its other tenants), so this is the host side one "
                           f"GPU's job actually gets"),
            "c1_full": {"seconds": round(c1_s, 4), "GBs": round(1024 * 4096 * esize / c1_s / 1e9, 4)},
            "extrapolated_seconds": round(total_s, 2), "shapes_sampled": len(lines),
            "sample": (f"oracle/awq_oracle.c ({'clip search ' + str(search) + ', ' if search else ''}"
                       f"bit-exact restatement of awq.py, OpenMP over rows, {threads} "
                       f"threads = the box's CPU share OMP_NUM_THREADS; node shows {node} CPUs) - C1 in full, "
                       f"then row samples of every {workload} shape ({'; '.join(lines)}; "
                       f"{sampled / 1e9:.2f} GB sampled), EXTRAPOLATED by row count and multiplicity to the whole "
                       f"set; {REFERENCE_CPU}")}


def packed_out_shapes(shape, bits, gs):
    """qweight / qzeros / scales shapes and dtypes of one tensor's packed outputs (PackedBatch)."""
    rows = 1 if len(shape) <= 1 else shape[0]
    K = int(torch.Size(shape).numel()) // rows
    G, per = -(-K // gs), 32 // bits
    return {"qweight": ((rows, -(-K // per)), torch.int32), "qzeros": ((rows, -(-G // per)), torch.int32),
            "scales": ((rows, G), torch.float16)}


def gather_leg(batch, rank, world, dev, backend, iters=2, shard_owner=None, all_shapes=None, bits=4, gs=128):
    """N>1 only, after the timed region: the CLI's exchange step (distributed.gather_to_rank0,
    zero-copy point-to-point into rank 0's outputs) on every rank's packed outputs of its shard (the real
    exchange of the CLI's torchrun mode; with --replica, of its replica).  Reported beside
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
    got = D.gather_to_rank0(local, owner, shapes, comm)               # warmup (connects the P2P channels)
    del got
    torch.cuda.synchronize(dev)
    D.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        got = D.gather_to_rank0(local, owner, shapes, comm)
        del got
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
    return {"what": what + f", batched P2P straight into rank 0's output tensors ({backend}); outside the timed region",
            "bytes_to_rank0": moved, "ms": round(t * 1e3, 3), "GBs_into_rank0": round(moved / t / 1e9, 2)}


def write_leg(batch, rank, dev, out_dir, chunk_size=10):
    """The CLI's per-rank output step (torchrun mode, --dist_output per_rank) on this rank's
    packed results: D2H into pinned memory, then chunk files written by main.ChunkWriter
    under the rank's private stem.  Outside the timed region; max over ranks."""
    import shutil
    from awq_quantizer import distributed as D
    from awq_quantizer.main import ChunkWriter, _rank_stem
    d = os.path.join(out_dir, f"bench_write_rank{rank:05d}")
    os.makedirs(d, exist_ok=True)
    torch.cuda.synchronize(dev)
    D.barrier()
    t0 = time.perf_counter()
    res = batch.results()
    host = {}
    for n in batch.names:
        host[n] = {f: (v.to("cpu", non_blocking=True) if isinstance(v, torch.Tensor) and v.is_cuda else v)
                   for f, v in res[n].items()}
    torch.cuda.synchronize(dev)
    t_d2h = time.perf_counter() - t0
    w = ChunkWriter(list(batch.names), d, chunk_size, False, stem=_rank_stem(rank), metadata=False)
    for n in batch.names:
        w.done(n, host[n])
    w.close()
    os.sync()
    t = time.perf_counter() - t0
    nbytes = sum(os.path.getsize(os.path.join(d, f)) for f in os.listdir(d))
    t_max = D.max_over_ranks(t, dev)
    shutil.rmtree(d, ignore_errors=True)
    return {"what": "per-rank output: D2H of the rank's packed shard + chunk files (main.ChunkWriter, torch.save) "
                    "+ sync; outside the timed region",
            "bytes_rank0": nbytes, "chunks_rank0": w.n_chunks, "d2h_s_rank0": round(t_d2h, 4),
            "s_rank0": round(t, 4), "s_max_over_ranks": round(t_max, 4), "GBs_rank0": round(nbytes / t / 1e9, 3)}


KERNEL_SOURCES = ("awq-converter_amd/csrc/awq_fast.hip", "awq-converter_amd/csrc/awq_quant.h",
                  "awq-converter_amd/csrc/awq_internal.h")


def kernel_source_hash(sources=KERNEL_SOURCES):
    """sha256 of a kernel's sources (what a recorded PMC figure is valid for)."""
    import hashlib
    h = hashlib.sha256()
    for p in sources:
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def recorded_traffic(path, key):
    """HBM traffic per launch recorded by a separate rocprofv3 --pmc run of this same
    command (scripts/profile_round.sh -> scripts/pmc_traffic.py; FETCH_SIZE x2 gfx950
    correction).  Counters cannot be read in-process, so the field is a RECORDED figure,
    labelled with its file, the commit and the kernel-source hash it was measured on; when
    the streaming kernel's sources have changed since, it is marked stale and `traffic`
    is null."""
    try:
        with open(path) as f:
            rec = json.load(f).get(key)
    except (OSError, ValueError):
        return None, None
    if not rec:
        return None, None
    now = kernel_source_hash()
    stale = rec.get("kernel_source_sha256") != now
    src = {"file": os.path.relpath(path, ROOT), "key": key, "commit": rec.get("commit"), "date": rec.get("date"),
           "kernel_source_sha256": rec.get("kernel_source_sha256"), "kernel_source_sha256_now": now,
           "stale": stale, "traffic_over_algorithmic": rec.get("traffic_over_algorithmic"),
           "note": "recorded by a separate rocprofv3 --pmc pass (FETCH_SIZE x2 + WRITE_SIZE), not this run"}
    return (None if stale else rec.get("hbm_bytes_per_launch")), src


# VALU issue ceiling: one VALU issue slot per SIMD per quad-cycle (4 cycles), 256 CUs x 4
# SIMDs at the 2.4 GHz max clock = 614.4 G slots/s.  A slot issues one VALU instruction, or
# two of the dual-issue class (plain f32 add / sub / mul / fma, f16 mul, v_mov / v_and /
# v_add_u32); conversions, v_rndne, v_med3 / v_max / v_min, DPP, packed f32 / f16, v_fma_mix
# and shifts take a slot each, v_exp / v_rcp two (scripts/valu_probe.hip + valu_classes.py,
# profiles/round5/r5k/valu_classes.json: SQ_ACTIVE_INST_VALU counts a kernel's slot-quads
# per instruction, SQ_ACTIVE_INST_VALU2 the quads that issued two).  A VALU-bound kernel's
# peak rate of work units = 614.4 G / its issue slots per unit, (SQ_ACTIVE_INST_VALU -
# SQ_ACTIVE_INST_VALU2) / units, recorded by a rocprofv3 --pmc pass of this same command
# (scripts/pmc_valu.py); frac is then the share of the chip's VALU issue slots the kernel keeps
# busy.  (The guide's 157.3 TFLOP/s fp32 vector peak is the dual-issued / packed FMA rate:
# 2 cycles per 64-lane instruction, reached only by a stream of dual-issue-class instructions.)
VALU_SLOT_RATE = 256 * 4 * 2.4e9 / 4
ACT_SOURCES = ("awq-converter_amd/csrc/awq_actsearch.hip", "awq-converter_amd/csrc/awq_refmath.h",
               "awq-converter_amd/csrc/awq_internal.h")


def recorded_valu(path, key, sources):
    """VALU issue slots per unit recorded for `key` (scripts/pmc_valu.py), None when absent,
    recorded without the dual-issue counter, or recorded on other kernel sources (stale)."""
    try:
        with open(path) as f:
            rec = json.load(f).get(key)
    except (OSError, ValueError):
        return None, None
    if not rec:
        return None, None
    now = kernel_source_hash(sources)
    stale = rec.get("kernel_source_sha256") != now
    src = {"file": os.path.relpath(path, ROOT), "key": key, "commit": rec.get("commit"), "date": rec.get("date"),
           "kernel_source_sha256": rec.get("kernel_source_sha256"), "kernel_source_sha256_now": now, "stale": stale,
           "counters": {k: rec[k] for k in ("valu_insts_per_dispatch", "valu_lane_instr_per_unit",
                                              "dual_issued_instr_frac", "valu_slot_occupancy",
                                              "effective_clock_ghz") if k in rec},
           "note": "recorded by a separate rocprofv3 --pmc pass (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, "
                   "SQ_ACTIVE_INST_VALU2, GRBM_GUI_ACTIVE) of this command, not this run"}
    return (None if stale else rec.get("valu_slots_per_unit")), src


def valu_roofline(units, kern_s, per_unit, src, unit_name):
    """roofline object of a VALU-bound kernel: achieved units/s against the VALU issue-slot
    ceiling for its own slots per unit."""
    achieved = units / kern_s / 1e9
    peak = VALU_SLOT_RATE / per_unit / 1e9 if per_unit else None
    r = {"bound": "valu", "achieved": round(achieved, 2), "peak": round(peak, 2) if peak else None,
         "unit": f"G {unit_name}/s", "frac": round(achieved / peak, 4) if peak else None, "traffic": None,
         "units_per_launch": units, "valu_slots_per_unit": per_unit, "valu_slot_rate_per_s": VALU_SLOT_RATE,
         "peak_basis": "MI355X VALU issue slots (256 CU x 4 SIMD x 2.4 GHz / 4 cycles = 614.4 G slots/s; a slot "
                       "issues one VALU instruction or two of the dual-issue class) / the kernel's slots per unit "
                       "((SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / units)"}
    if src:
        r["valu_source"] = src
        # the same rate against the all-dual-issue ceiling (2 cycles per 64-lane instruction,
        # the guide's 157.3 TFLOP/s fp32 vector figure): how far the instruction MIX is from a
        # stream that pairs every instruction — not an issue-slot fraction
        lane = (src.get("counters") or {}).get("valu_lane_instr_per_unit")
        if lane and not src.get("stale"):
            dual_peak = 256 * 4 * 64 / 2 * 2.4e9 / lane / 1e9
            r["frac_of_dual_issue_rate"] = round(achieved / dual_peak, 4)
    return r


def add_valu_floor(roof, kind, dtype_name, bits, symmetric):
    """The algorithmic floor beside the issue-slot roofline (scripts/valu_floor.py ->
    profiles/round6/valu_floor.json): the per-candidate-element instruction chain the
    reference's per-op rounding forces, priced in issue slots.  floor_frac = achieved rate /
    (614.4 G slots/s / floor slots per unit); slots_over_floor = the kernel's recorded slots
    per unit / the floor's."""
    key = f"{kind}.{dtype_name}.{'sym' if symmetric else 'asym'}"
    path = os.path.join(ROOT, "profiles", "round6", "valu_floor.json")
    try:
        with open(path) as f:
            rec = json.load(f).get(key) if bits == 4 else None
    except (OSError, ValueError):
        rec = None
    if not rec:
        roof["floor_slots_per_unit"] = None
        roof["floor_note"] = f"no floor derived for {key} at {bits} bits (scripts/valu_floor.py)"
        return
    fl = rec["floor_slots_per_unit"]
    floor_peak = VALU_SLOT_RATE / fl / 1e9
    roof["floor_slots_per_unit"] = fl
    roof["floor_peak"] = round(floor_peak, 2)
    roof["floor_frac"] = round(roof["achieved"] / floor_peak, 4)
    if roof.get("valu_slots_per_unit"):
        roof["slots_over_floor"] = round(roof["valu_slots_per_unit"] / fl, 3)
    roof["floor_source"] = {"file": os.path.relpath(path, ROOT), "key": key,
                            "floor_slots_per_element": rec["floor_slots_per_element"],
                            "excess_instructions_by_type": rec.get("excess_instructions_by_type")}


def main():
    args = parse()
    if args.mode == "act":
        return main_act(args)
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

    shard = not args.replica
    all_shapes = shapes_of(args.workload)
    dtype = DTYPES[args.dtype]
    esize = torch.empty((), dtype=dtype).element_size()
    if shard:
        # strong scaling: rank r quantizes the tensors LPT assigns it (tensor i is seeded by
        # its index, so the data do not depend on the world size)
        owner = D.shard([int(torch.Size(s).numel()) for s in all_shapes], world)
        mine = [i for i in range(len(all_shapes)) if owner[i] == rank]
    else:
        owner = None
        mine = list(range(len(all_shapes)))
    shapes = [all_shapes[i] for i in mine]
    elems = sum(int(torch.Size(s).numel()) for s in shapes)
    total_elems = sum(int(torch.Size(s).numel()) for s in all_shapes)
    in_bytes = elems * esize
    # bytes all ranks quantize per step: the whole set once (shard) or one replica per rank
    step_bytes = total_elems * esize if shard else in_bytes * world
    reps = args.replicas or max(1, -(-(1 << 30) // max(1, in_bytes)))   # >= 1 GiB of inputs in rotation
    stream = torch.cuda.current_stream(dev)
    # the same ceiling at the footprint this rank streams (its inputs, up to 128 GiB), before
    # the set is allocated: a 1 GiB buffer runs the structure ~1.5 % faster than a 128 GiB one
    # (profiles/round2/r2g_mix_probe_sizes.log), and the kernel streams 141 GB
    ceiling_fp, fp_bytes = None, 0
    if not args.no_copy_ceiling and in_bytes >= (4 << 30):
        fp_bytes = min(in_bytes // (1 << 30), 128) << 30
        ceiling_fp = stream_ceiling(dev, stream, args.clock_warm_ms, nbytes=fp_bytes, iters=5)
        torch.cuda.empty_cache()
    batches = []
    for r in range(reps):
        if shard:
            inputs = make_set(all_shapes, r * 100003, dev, dtype, only=set(mine))
        else:
            inputs = make_set(shapes, (rank * 64 + r) * 100003, dev, dtype)
        search = (args.search_grid, args.search_candidates) if args.mode == "search" else None
        batches.append(PackedBatch(inputs, bits=args.bits, symmetric=args.symmetric, parity=args.parity,
                                   group_size=args.group_size, search=search))
        del inputs
    torch.cuda.synchronize()
    algo_bytes = batches[0].algorithmic_bytes()

    barrier = D.barrier
    # clock warm-up on every rank (and the ceiling figure) before the warmup launches
    ceiling = None if args.no_copy_ceiling else stream_ceiling(dev, stream, args.clock_warm_ms)
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

    elapsed = D.max_over_ranks(elapsed, dev)
    kern_max_s = D.max_over_ranks(kern_avg_s, dev)
    per_rank = D.all_gather_floats([kern_avg_s * 1e6, float(elems)], dev)   # [kernel us, elements] by rank
    del batches[1:]
    torch.cuda.empty_cache()
    gather = (gather_leg(batches[0], rank, world, dev, backend, shard_owner=owner,
                         all_shapes=all_shapes, bits=args.bits, gs=args.group_size)
              if world > 1 and not args.no_gather else None)

    written = write_leg(batches[0], rank, dev, args.write_dir) if args.write_dir else None

    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    value = step_bytes * args.steps / elapsed / 1e9
    achieved = algo_bytes / kern_avg_s / 1e9
    key = f"{args.workload}.b{args.bits}.{'sym' if args.symmetric else 'asym'}.{'parity' if args.parity else 'packed'}"
    if args.group_size != 128:
        key += f".gs{args.group_size}"
    if args.dtype != "bf16":
        key += f".{args.dtype}"
    if args.mode == "search":
        key += f".search{args.search_candidates}of{args.search_grid}"
    if world > 1:
        key += f".{'shard' if shard else 'replica'}{world}"
    traffic, traffic_src = recorded_traffic(args.traffic_json, key)
    metric = METRIC.replace("group_size=128", f"group_size={args.group_size}").replace("bf16", args.dtype)
    if args.mode == "search":
        metric = metric.replace(", 1/2/4/8", f" with the clip search ({args.search_candidates} of "
                                             f"{args.search_grid} candidates), 1/2/4/8").replace("% HBM roofline",
                                                                                             "% VALU roofline")
    line = {
        "metric": metric,
        "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong" if shard else "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
        "config": {"workload": f"{args.workload}: {DESCR[args.workload]}", "tensors": len(all_shapes),
                   "elements": total_elems, "group_size": args.group_size, "bits": args.bits, "symmetric": args.symmetric,
                   "outputs": "qweight+qzeros+fp16 scales" + (" + int32 tensor_q/zero_points" if args.parity else ""),
                   "launches_per_step": 1, "input_replicas_rotated": reps,
                   "parallelism": (f"shard{world} (ONE copy of the set, tensor list LPT-sharded over the ranks; "
                                   f"rank 0 holds {len(shapes)} tensors, {elems} elements)") if shard else
                                  f"replica{world} (each rank quantizes its own replica of the tensor set)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "kernel_avg_us": round(kern_avg_s * 1e6, 2),
                     "kernel_avg_us_max_over_ranks": round(kern_max_s * 1e6, 2),
                     "timing": f"hip events ({args.events}) on the launch stream, rank 0's launches"},
    }
    if traffic_src:
        line["roofline"]["traffic_source"] = traffic_src
    if args.mode == "search":
        # VALU-bound: candidate-elements (elements x candidates) against the VALU issue ceiling;
        # the HBM view of the same launch stays beside it
        hbm = line.pop("roofline")
        per_unit, vsrc = recorded_valu(args.valu_json, key, KERNEL_SOURCES)
        line["roofline"] = valu_roofline(elems * args.search_candidates, kern_avg_s, per_unit, vsrc,
                                         "candidate-elements")
        line["roofline"]["kernel_avg_us"] = hbm["kernel_avg_us"]
        line["roofline"]["timing"] = hbm["timing"]
        line["roofline"]["hbm_view"] = {k: hbm[k] for k in ("achieved", "peak", "unit", "frac", "traffic",
                                                            "algorithmic_bytes_per_launch") if k in hbm}
        add_valu_floor(line["roofline"], "search", args.dtype, args.bits, args.symmetric)
        line["config"]["search"] = {"grid": args.search_grid, "candidates": args.search_candidates,
                                    "alpha": f"1 - i/{args.search_grid}, i < {args.search_candidates}"}
    if world > 1:       # the LPT shard's balance: per-rank kernel time and elements
        ku = [r[0] for r in per_rank]
        el = [int(r[1]) for r in per_rank]
        line["ranks"] = {"kernel_avg_us": [round(v, 2) for v in ku], "elements": el,
                         "kernel_max_over_min": round(max(ku) / max(min(ku), 1e-9), 4),
                         "elements_max_over_min": round(max(el) / max(min(el), 1), 4)}
    if gather:
        line["exchange"] = gather
    if written:
        line["write"] = written
    if ceiling:
        # read_dominant_ceiling: at the streamed footprint when the set is >= 4 GiB, else 1 GiB
        ref = ceiling_fp or ceiling
        hv = line["roofline"].get("hbm_view", line["roofline"])
        hv["read_dominant_ceiling"] = round(ref, 1)
        hv["frac_of_ceiling"] = round(achieved / ref, 4)
        hv["ceiling_footprint_bytes"] = fp_bytes if ceiling_fp else 1 << 30
        hv["read_dominant_ceiling_1gib"] = round(ceiling, 1)
        hv["frac_of_ceiling_1gib"] = round(achieved / ceiling, 4)
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(args.workload, args.cpu_sample_seconds, args.group_size, dtype,
                                            search=(args.search_grid, args.search_candidates)
                                            if args.mode == "search" else None)
    print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


# one Llama-3-8B decoder block: layer group -> (rows of the linears reading the same input, in_features)
ACT_BLOCK = {"qkv": ([4096, 1024, 1024], 4096), "o": ([4096], 4096), "gate_up": ([14336, 14336], 4096),
             "down": ([4096], 14336)}


def act_cpu_baseline(budget_s, n_grid, tokens, dtype, bits, symmetric, gs):
    """The oracle's activation-aware search (oracle_act_*, OpenMP over rows) on a row sample of
    the block's o_proj group, rate in weight bytes / s (the oracle restates the product's own
    definition: the reference has no such search)."""
    from oracle import awq_oracle as orc
    threads, node, aff = host_cpus()
    orc.set_threads(threads)
    g = torch.Generator().manual_seed(7)
    K = 4096
    esize = torch.empty((), dtype=dtype).element_size()
    x = (torch.randn(tokens, K, generator=g) * 2).to(dtype)
    rows, t, reps = 64, 0.0, 0
    w = (torch.randn(rows, K, generator=g) * 0.02).to(dtype)
    orc.awq_search([w], x, n_grid=n_grid, group_size=gs, bits=bits, symmetric=symmetric)     # warm
    while reps < 2 or (t < budget_s and reps < 100):
        t0 = time.perf_counter()
        orc.awq_search([w], x, n_grid=n_grid, group_size=gs, bits=bits, symmetric=symmetric)
        t += time.perf_counter() - t0
        reps += 1
    return {"value": round(rows * K * esize * reps / t / 1e9, 6), "unit": "GB/s", "cores": threads, "kind": "port",
            "node_cpus": node, "affinity_cpus": aff,
            "sample": (f"oracle/awq_oracle.c oracle_act_* (the product's definition restated; OpenMP over rows, "
                       f"{threads} threads = the box's CPU share) on a {rows}x{K} slice of o_proj with {tokens} "
                       f"tokens x {n_grid} candidates, {reps} runs in {t:.1f} s; rate in weight bytes")}


def main_act(args):
    """--mode act: the activation-aware search (scale_method="awq", AWQQuantizer.quantize_layer_group)
    of one Llama-3-8B block — q/k/v, o, gate/up, down, each with its own synthetic calibration
    input (tokens x in_features, 1/32 of the channels x30: salient channels).  A step = all four
    layer groups: statistics, w_mean, scale table, the loss kernel over every candidate, select,
    W·diag(s) and its packed quantization.  value = the block's weight bytes per second.  The
    loss kernel (act_loss_kernel, ~all of the search's time) is then timed alone on the same
    inputs and quoted against the VALU issue ceiling.  N > 1: every rank its own block (weak)."""
    from awq_quantizer import _hip
    from awq_quantizer import distributed as D
    from awq_quantizer.quantization import AWQQuantizer
    backend = os.environ.get("AWQ_DIST_BACKEND", "nccl")
    rank, local, world = D.init(backend)
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    _hip.require_device(dev)
    dtype = DTYPES[args.dtype]
    esize = torch.empty((), dtype=dtype).element_size()
    n_grid, gs = args.search_grid, args.group_size
    q = AWQQuantizer(bits=args.bits, group_size=gs, symmetric=args.symmetric, scale_method="awq", search_grid=n_grid,
                     device=str(dev), logger_level="ERROR")
    groups = []
    for gi, (gname, (rows, K)) in enumerate(ACT_BLOCK.items()):
        g = torch.Generator(device=dev).manual_seed(1000 * rank + gi)
        ws = {f"{gname}.{j}": (torch.randn(r, K, device=dev, generator=g) * 0.02).to(dtype) for j, r in enumerate(rows)}
        amp = torch.ones(K, device=dev)
        amp[torch.randperm(K, generator=g, device=dev)[: K // 32]] = 30.0
        x = (torch.randn(args.act_tokens, K, device=dev, generator=g) * amp).to(dtype)
        groups.append((ws, x))
    elems = sum(w.numel() for ws, _ in groups for w in ws.values())
    cand = elems * n_grid
    stream = torch.cuda.current_stream(dev)

    def step():
        return [q.quantize_layer_group(ws, x) for ws, x in groups]

    if not args.no_copy_ceiling:
        stream_ceiling(dev, stream, args.clock_warm_ms)           # clock warm-up, as the main bench
    for _ in range(max(1, args.warmup)):
        res = step()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    D.barrier()
    elapsed = D.max_over_ranks(time.perf_counter() - t0, dev)
    best = [r["best"] for r in res]
    # the loss kernel alone: same weights, statistics, table and reciprocal table
    prep = []
    for ws, x in groups:
        wl = list(ws.values())
        xm, xs = _hip.act_stats(x)
        table = _hip.act_scale_table(xm, _hip.weight_mean(wl, gs), n_grid)
        prep.append((wl, xs, table, _hip.act_recip_table(table)))
    for wl, xs, table, rt in prep:
        _hip.act_search_losses(wl, xs, table, gs, args.bits, args.symmetric, rtable=rt)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(args.steps):
        for wl, xs, table, rt in prep:
            _hip.act_search_losses(wl, xs, table, gs, args.bits, args.symmetric, rtable=rt)
    b.record(stream)
    torch.cuda.synchronize()
    loss_s = a.elapsed_time(b) / 1e3 / args.steps                 # all loss launches of one step
    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    key = f"act.llama3-8b-block.t{args.act_tokens}.g{n_grid}.{args.dtype}.b{args.bits}.{'sym' if args.symmetric else 'asym'}"
    per_unit, vsrc = recorded_valu(args.valu_json, key, ACT_SOURCES)
    roof = valu_roofline(cand, loss_s, per_unit, vsrc, "candidate-elements")
    add_valu_floor(roof, "act", args.dtype, args.bits, args.symmetric)
    roof.update({"kernel": "act_loss_kernel (7 launches per step: one per linear)",
                 "kernel_avg_us": round(loss_s / len([w for ws, _ in groups for w in ws]) * 1e6, 2),
                 "loss_kernels_us_per_step": round(loss_s * 1e6, 2),
                 "loss_share_of_step": round(loss_s / (elapsed / args.steps), 4),
                 "timing": "hip events around the step's 7 loss launches (same inputs), repeated --steps times"})
    wbytes = elems * esize
    line = {"metric": (f"{args.dtype} GB/sec of Llama-3-8B block weights through the activation-aware search "
                       f"({args.act_tokens} tokens x {n_grid} candidates, group_size={gs}) + packed quantization, "
                       f"1 MI355X per block; % VALU roofline of the loss kernel"),
            "value": round(wbytes * world * args.steps / elapsed / 1e9, 3), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (weights N(0, 0.02); activations N(0, 1) with 1/32 of the channels x30)",
            "config": {"workload": "llama3-8b block: q/k/v, o, gate/up, down layer groups", "tensors": 7,
                       "elements": elems, "tokens": args.act_tokens, "candidates": n_grid, "group_size": gs,
                       "bits": args.bits, "symmetric": args.symmetric, "duo_scaling": True, "best_ratio": best,
                       "parallelism": f"replica{world} (every rank its own block)"},
            "roofline": roof}
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = act_cpu_baseline(min(args.cpu_sample_seconds, 15.0), n_grid, args.act_tokens, dtype,
                                                args.bits, args.symmetric, gs)
    print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
