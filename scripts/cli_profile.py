#!/usr/bin/env python3
"""CLI end to end on BASELINE configs 3 / 4 (the reference's own flow, main.py:515-676):
synthetic multi-file safetensors checkpoints with the exact tensor shapes of opt-350m
(3 files) and Llama-3-8B (4 files), quantized by awq_quantizer.main.main() to the reference
chunk format and to the packed format.  Per run: wall time, GB/s of input, the CLI's phase
times; run 0 is the process's first call (HIP / library / pinned-pool warm-up inside it),
`--evict` first drops the checkpoint from the page cache (posix_fadvise DONTNEED: a disk
read).  Then the ceilings the pipeline runs against, measured in the same process: pinned
host -> HBM (hipMemcpyAsync via torch, 1 GiB blocks), HBM -> pinned, and page cache ->
pinned host with the CLI's reader-thread count (pread).

  python scripts/cli_profile.py --workload llama3-8b --shards 4 --formats packed,reference
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd"), os.path.join(ROOT, "scripts")]
import torch  # noqa: E402

import cli_bench  # noqa: E402


def evict(model_dir):
    for f in os.listdir(model_dir):
        p = os.path.join(model_dir, f)
        fd = os.open(p, os.O_RDONLY)
        try:
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        finally:
            os.close(fd)


def probes(model_dir, threads):
    dev = torch.device("cuda", 0)
    n = 1 << 30
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    out = {}
    for name, (dst, src) in {"h2d_pinned_GBs": (d, h), "d2h_pinned_GBs": (h, d)}.items():
        with torch.cuda.stream(s):
            dst.copy_(src, non_blocking=True)
        s.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for _ in range(8):
                dst.copy_(src, non_blocking=True)
        s.synchronize()
        out[name] = round(8 * n / (time.perf_counter() - t0) / 1e9, 2)
    # D2H into a large pinned destination walked once (the reference format's per-chunk output
    # buffers: tens of GB, each page written once) vs the same 1 GiB reused above
    big = torch.empty(8 * n, dtype=torch.uint8, pin_memory=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        for k in range(8):
            big[k * n:(k + 1) * n].copy_(d, non_blocking=True)
    s.synchronize()
    out["d2h_pinned_8GiB_walk_GBs"] = round(8 * n / (time.perf_counter() - t0) / 1e9, 2)
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        for k in range(8):
            big[k * n:(k + 1) * n].copy_(d, non_blocking=True)
    s.synchronize()
    out["d2h_pinned_8GiB_second_walk_GBs"] = round(8 * n / (time.perf_counter() - t0) / 1e9, 2)
    del big
    # both directions at once on two streams (the native pipeline's H2D and D2H overlap)
    h2, d2, s2 = torch.empty_like(h).pin_memory(), torch.empty_like(d), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(8):
        with torch.cuda.stream(s):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()
    out["h2d_plus_d2h_concurrent_GBs"] = round(16 * n / (time.perf_counter() - t0) / 1e9, 2)
    del h2, d2
    # page cache -> pinned (the CLI's read path): every file, `threads` preads in flight
    files = [os.path.join(model_dir, f) for f in sorted(os.listdir(model_dir)) if f.endswith(".safetensors")]
    total = sum(os.path.getsize(f) for f in files)
    for f in files:       # warm the page cache
        with open(f, "rb") as fh:
            while fh.read(1 << 26):
                pass
    blk = 64 << 20
    bufs = [torch.empty(blk, dtype=torch.uint8, pin_memory=True) for _ in range(threads)]
    jobs = [(f, off) for f in files for off in range(0, os.path.getsize(f), blk)]

    def rd(i, job):
        f, off = job
        fd = os.open(f, os.O_RDONLY)
        try:
            return os.preadv(fd, [memoryview(bufs[i % threads].numpy())], off)
        finally:
            os.close(fd)
    with ThreadPoolExecutor(threads) as pool:
        t0 = time.perf_counter()
        got = sum(pool.map(rd, range(len(jobs)), jobs))
        out["pagecache_to_pinned_GBs"] = round(got / (time.perf_counter() - t0) / 1e9, 2)
    out["pread_threads"] = threads
    out["checkpoint_GB"] = round(total / 1e9, 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="opt-350m")
    ap.add_argument("--shards", type=int, default=3)
    ap.add_argument("--formats", default="packed,reference")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--evict", action="store_true", help="run 0 of the first format reads from disk")
    ap.add_argument("--cprofile", default=None, help="cProfile the last run's pipeline thread to this file")
    ap.add_argument("--extra", default="", help="extra CLI flags")
    ap.add_argument("--engines", default="native", help="--stream_engine values to run, e.g. native,python")
    ap.add_argument("--stream-opts", default="", help="'/'-separated settings of main.STREAM_OPTS to run the "
                    "native engine under, each 'default' or k=v[,k=v] over slot_bytes / nslots / copy_streams, "
                    "e.g. default/copy_streams=1/slot_bytes=536870912")
    args = ap.parse_args()
    from awq_quantizer import main as cli_mod
    work = args.workdir or tempfile.mkdtemp(prefix="awq_cli_")
    model = os.path.join(work, f"model_{args.workload}_{args.shards}")
    os.makedirs(model, exist_ok=True)
    t0 = time.time()
    nbytes = cli_bench.build_model(model, args.workload, args.shards)
    print(json.dumps({"workload": args.workload, "files": args.shards, "input_GB": round(nbytes / 1e9, 3),
                      "build_s": round(time.time() - t0, 1)}), flush=True)
    first = True
    opts_list = [{} if o == "default" else {k: int(v) for k, v in (kv.split("=") for kv in o.split(","))}
                 for o in args.stream_opts.split("/") if o.strip()] or [{}]
    combos = [(f, e, o) for f in args.formats.split(",") for e in args.engines.split(",")
              for o in (opts_list if e == "native" else [{}])]
    for fmt, eng, opts in combos:
        cli_mod.STREAM_OPTS.clear()
        cli_mod.STREAM_OPTS.update(opts)
        for r in range(args.runs):
            if first and args.evict:
                evict(model)
            out = os.path.join(work, f"out_{fmt}_{r}")
            cli_mod.TIMINGS.clear()
            argv = ["--model_id", model, "--output_dir", out, "--log_level", "WARNING",
                    "--output_format", fmt, "--stream_engine", eng] + args.extra.split()
            t0 = time.perf_counter()
            if args.cprofile and r == args.runs - 1:
                import cProfile
                prof = cProfile.Profile()
                rc = prof.runcall(cli_mod.main, argv)
                prof.dump_stats(args.cprofile + f".{fmt}.{eng}")
            else:
                rc = cli_mod.main(argv)
            wall = time.perf_counter() - t0
            assert rc == 0
            ob = sum(os.path.getsize(os.path.join(out, f)) for f in os.listdir(out))
            print(json.dumps({"workload": args.workload, "format": fmt, "engine": eng, "opts": opts, "run": r,
                              "kind": ("process-first" + (", page cache evicted" if args.evict else "")) if first
                              else "warm", "input_GB": round(nbytes / 1e9, 3), "output_GB": round(ob / 1e9, 3),
                              "wall_s": round(wall, 4), "input_GBs": round(nbytes / wall / 1e9, 3),
                              "phases": cli_mod.TIMINGS}, default=str), flush=True)
            first = False
            shutil.rmtree(out, ignore_errors=True)
    print(json.dumps({"ceilings": probes(model, 16)}), flush=True)
    if args.cprofile:
        import pstats
        for fmt, eng in [(f, e) for f in args.formats.split(",") for e in args.engines.split(",")]:
            p = args.cprofile + f".{fmt}.{eng}"
            if os.path.exists(p):
                print(f"--- cProfile {fmt} {eng} (pipeline thread, last run) ---")
                pstats.Stats(p).sort_stats("cumulative").print_stats(30)
                pstats.Stats(p).sort_stats("tottime").print_stats(25)
    if args.workdir is None:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
