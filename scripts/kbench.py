#!/usr/bin/env python3
"""Kernel-level bench for tuning: per-launch time of the ragged quantize kernel on several
tensor sets, for one or more library builds (--lib) and grid caps (--blocks), interleaved
in ONE process (guide §5.4 rule 24).  Prints a table + JSON lines.

  python scripts/kbench.py --sets opt-125m,llama3-8b-mlp --blocks 0,1536 --libs a.so,b.so
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402

import bench  # noqa: E402  (shape manifests)

SETS = dict(bench.WORKLOADS)
SETS["llama3-8b-mlp"] = [((14336, 4096), 8), ((4096, 14336), 4)]      # 705 M elements
SETS["c1x64"] = [((1024, 4096), 64)]
SETS["k768"] = [((50272, 768), 4)]
SETS["falcon7b-mlp"] = [((18176, 4544), 8), ((4544, 18176), 4)]   # K = 4544: padded rows at gs 128
SETS["qwen05-odd"] = [((4864, 896), 8), ((151936, 896), 1)]   # K = 896: 7 groups (odd) at gs 128 -> word tiles (2 rows per tile)
SETS.setdefault("c1", [((1024, 4096), 1)])
SETS["lm-head-8b"] = [((128256, 4096), 1)]          # one large tensor per launch (quantize_packed per tensor)
SETS["down-8b"] = [((4096, 14336), 1)]


def shapes_of(name):
    out = []
    for s, c in SETS[name]:
        out += [s] * c
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", default="opt-125m,c1x64,llama3-8b-mlp,k768")
    ap.add_argument("--libs", default="")
    ap.add_argument("--blocks", default="0")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--symmetric", action="store_true")
    ap.add_argument("--parity", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "f32"])
    ap.add_argument("--group-size", type=int, default=128)
    ap.add_argument("--search", type=int, default=0, help="clip-search candidates of 20 (0 = RTN): "
                    "awq_quantize_ragged_search")
    ap.add_argument("--arena", action="store_true",
                    help="inputs as views of ONE device buffer per replica instead of one allocation per tensor")
    args = ap.parse_args()
    from awq_quantizer import _hip
    from awq_quantizer.quantization.batch import PackedBatch
    dev = torch.device("cuda", 0)
    libs = [p for p in args.libs.split(",") if p] or [_hip.LIB_PATH]
    handles = {}
    for p in libs:
        lib = ctypes.CDLL(os.path.abspath(p))
        for name, (res, argt) in _hip.SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is not None:
                fn.restype = res
                fn.argtypes = argt
        if lib.awq_abi_version() < 5:   # older builds: no group_size argument (gs 128 only)
            lib.awq_quantize_ragged.argtypes = _hip.SIGNATURES["awq_quantize_ragged"][1][:-3] + [ctypes.c_void_p]
        elif lib.awq_abi_version() < 7:   # no flags argument
            lib.awq_quantize_ragged.argtypes = _hip.SIGNATURES["awq_quantize_ragged"][1][:-2] + [ctypes.c_void_p]
        handles[p] = lib
    _hip.load_library()
    _hip.require_device(dev)

    # copy ceiling: 1 GiB bf16 copy (read 1 GiB + write 1 GiB)
    a = torch.empty(1 << 29, dtype=torch.bfloat16, device=dev).normal_()
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    copy_gbs = 2 * a.numel() * 2 * 10 / (e0.elapsed_time(e1) / 1e3) / 1e9
    print(json.dumps({"copy_ceiling_GBs": round(copy_gbs, 1)}))
    del a, b

    batches = {}
    for sname in args.sets.split(","):
        shapes = shapes_of(sname)
        nbytes = sum(int(torch.Size(s).numel()) * (4 if args.dtype == "f32" else 2) for s in shapes)
        reps = max(1, -(-(1 << 30) // nbytes))
        bl = []
        for r in range(reps):
            g = torch.Generator(device=dev)
            inputs = {}
            dt = {"f16": torch.float16, "f32": torch.float32}.get(args.dtype, torch.bfloat16)
            arena, off = None, 0
            if args.arena:
                arena = torch.empty(sum(-(-int(torch.Size(s).numel()) // 8) * 8 for s in shapes), dtype=dt, device=dev)
            for i, s in enumerate(shapes):
                g.manual_seed(r * 1000 + i)
                n = int(torch.Size(s).numel())
                t = arena[off:off + n].view(s) if arena is not None else torch.empty(s, dtype=dt, device=dev)
                off += -(-n // 8) * 8
                flat = t.view(s[0], -1) if len(s) > 1 else t.view(1, -1)
                step = max(1, (1 << 28) // flat.shape[1])
                for r0 in range(0, flat.shape[0], step):
                    blk = flat[r0:r0 + step]
                    blk.copy_(torch.randn(blk.shape, generator=g, device=dev) * 0.02)
                inputs[f"t{i}"] = t
            bl.append(PackedBatch(inputs, bits=args.bits, symmetric=args.symmetric, parity=args.parity,
                                  group_size=args.group_size))
        batches[sname] = bl
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    tables = {}

    def block_table(lp, lib, bt):
        """the per-workgroup tensor table planned by THIS library (its own workgroup size)"""
        key = (lp, id(bt))
        if key not in tables:
            arr = (_hip.TensorDesc * len(bt.descs))(*bt.descs)
            need = lib.awq_plan_block_tensor(arr, len(bt.descs), bt.total_tiles, None, 0)   # size query
            host = torch.empty(max(need, -(-bt.total_tiles // 4)), dtype=torch.int32)
            rc = lib.awq_plan_block_tensor(arr, len(bt.descs), bt.total_tiles, ctypes.c_void_p(host.data_ptr()),
                                           host.numel())
            assert rc > 0, lib.awq_last_error()
            tables[key] = host.to(dev)
        return tables[key]
    results = {}
    for rnd in range(args.rounds):
        for sname, bl in batches.items():
            for lp, lib in handles.items():
                for blk in args.blocks.split(","):
                    tun = _hip.Tuning()
                    if blk.startswith("t"):          # t<N>: non-persistent grid, N tiles per wave
                        tun.tiles_per_wave = int(blk[1:])
                    elif blk not in ("0", "nt"):     # nt: no per-block tensor table
                        tun.max_blocks = int(blk)
                    if hasattr(lib, "awq_set_tuning"):   # (csrc/awq_diag.h, diagnostics build; thread-local)
                        lib.awq_set_tuning(ctypes.byref(tun))
                    evs = []
                    for it in range(args.iters + 3):
                        bt = bl[it % len(bl)]
                        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        s0.record(stream)
                        table = None if blk == "nt" else block_table(lp, lib, bt).data_ptr()
                        abi = lib.awq_abi_version()
                        gsa = ((bt.group_size,) if abi >= 5 else ()) + ((bt.flags,) if abi >= 7 else ())
                        if args.search > 1:
                            rc = lib.awq_quantize_ragged_search(
                                ctypes.c_void_p(bt.descs_dev.data_ptr()), len(bt.descs), bt.total_tiles,
                                ctypes.c_void_p(table), _hip.AWQ_DTYPE[bt.dtype], bt.bits, int(bt.symmetric), *gsa,
                                20, args.search, ctypes.c_void_p(stream.cuda_stream))
                        else:
                            rc = lib.awq_quantize_ragged(ctypes.c_void_p(bt.descs_dev.data_ptr()), len(bt.descs),
                                                         bt.total_tiles, ctypes.c_void_p(table),
                                                         _hip.AWQ_DTYPE[bt.dtype], bt.bits, int(bt.symmetric),
                                                         *gsa, ctypes.c_void_p(stream.cuda_stream))
                        s1.record(stream)
                        assert rc == 0, lib.awq_last_error()
                        if it >= 3:
                            evs.append((s0, s1))
                    torch.cuda.synchronize()
                    us = [a.elapsed_time(b) * 1e3 for a, b in evs]
                    key = (sname, os.path.relpath(lp, ROOT) if os.path.isabs(lp) else lp, blk)
                    results.setdefault(key, []).append(statistics.median(us))
    for lib in handles.values():
        if hasattr(lib, "awq_set_tuning"):
            lib.awq_set_tuning(None)
    print(f"{'set':16s} {'lib':28s} {'blocks':>6s} {'us':>9s} {'algoGB/s':>9s} {'inGB/s':>8s} {'frac8T':>6s}")
    for (sname, lname, blk), v in results.items():
        bt = batches[sname][0]
        us = min(v)
        algo = bt.algorithmic_bytes() / (us / 1e6) / 1e9
        inp = bt.elements * bt.inputs[bt.names[0]].element_size() / (us / 1e6) / 1e9
        print(f"{sname:16s} {lname:28s} {blk:>6s} {us:9.1f} {algo:9.1f} {inp:8.1f} {algo / 8000:6.3f}")
        rec = {"set": sname, "lib": lname, "blocks": blk, "us": round(us, 2), "algo_GBs": round(algo, 1),
               "in_GBs": round(inp, 1), "rounds_us": [round(x, 1) for x in v]}
        if args.search > 1:
            rec["search_candidates"] = args.search
            rec["T_candidate_elements_per_s"] = round(bt.elements * args.search / (us / 1e6) / 1e12, 4)
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
