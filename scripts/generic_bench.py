#!/usr/bin/env python3
"""Throughput of the single-tensor entry point (awq_quantize_groups / awq_quantize_search)
per input dtype and group size: group sizes 32/64/128/256 take the streaming kernel, other
sizes <= 512 the row-segment kernel, larger ones (and fp64) the generic kernel.
--compare-generic runs every case a second time with tuning no_rowgroup=1 (generic kernel +
int32 staging + pack passes), interleaved in this process.

  python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16,f16,f32 --group-sizes 100,128
  python scripts/generic_bench.py --shape "1024,4096;4096,4096" --dtypes bf16   (";" separates shapes)
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402

DT = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32, "f64": torch.float64}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="14336,4096")
    ap.add_argument("--dtypes", default="bf16,f16,f32")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--search", type=int, default=0, help="clip-search candidates (0 = RTN)")
    ap.add_argument("--group-sizes", default="128")
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--compare-generic", action="store_true")
    ap.add_argument("--tunings", default="", help="'/'-separated awq_tuning settings to time the quantize under, "
                    "each 'default' or k=v[,k=v] (csrc/awq_diag.h, diagnostics build), e.g. default/rg_p1=1")
    ap.add_argument("--dequant", action="store_true", help="also time dequantize_packed of the packed result")
    ap.add_argument("--settle-ms", type=float, default=0.0,
                    help="stream this long (awq_stream_ceiling) before every timed loop: the clocks of a busy "
                         "chip (bench.py's ceiling probe does the same; an idle GPU's first ~5 ms run slower, "
                         "profiles/round6/r6h)")
    ap.add_argument("--dq-variants", default="1,3,6,7,8,9", help="--dq-ab: tuning dq_words_v1 values to time")
    ap.add_argument("--lib", default="", help="load this in-tree build instead of _lib/libawq_hip.so (A/B of builds)")
    ap.add_argument("--dq-ab", action="store_true", help="--dequant: also the round-2 word kernel (tuning dq_words_v1), "
                                                          "interleaved, 3 rounds")
    args = ap.parse_args()
    from awq_quantizer import _hip
    if args.lib:
        _hip.load_library(args.lib)
    dev = torch.device("cuda", 0)
    _hip.require_device(dev)
    for shape in args.shape.split(";"):
        for name in args.dtypes.split(","):
            for gs in (int(v) for v in args.group_sizes.split(",")):
                for generic in ((False, True) if args.compare_generic else (False,)):
                    for tun in (args.tunings.split("/") if args.tunings else ["default"]):
                        kw = {} if tun == "default" else {k: int(v) for k, v in (t.split("=") for t in tun.split(","))}
                        one(args, _hip, dev, shape, name, gs, generic, kw)


_settle_buf = {}


def settle(args, _hip, dev):
    """~args.settle_ms of streaming (1 GiB reads) so the timed loop starts at settled clocks."""
    if args.settle_ms <= 0:
        return
    import time
    if not _settle_buf:
        _settle_buf["src"] = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        _settle_buf["dst"] = torch.empty(1 << 28, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    t0 = time.time()
    while (time.time() - t0) * 1e3 < args.settle_ms:
        for _ in range(8):
            _hip.stream_ceiling(_settle_buf["src"], _settle_buf["dst"], st)
        torch.cuda.synchronize()


def one(args, _hip, dev, shape, name, gs, generic, tun=None):
    R, K = (int(v) for v in shape.split(","))
    G = -(-K // gs)
    per = 32 // args.bits
    g = torch.Generator(device=dev).manual_seed(R * 7919 + K * 31 + gs)   # same data in every process
    x = (torch.randn(R, K, device=dev, generator=g) * 0.02).to(DT[name])
    qw = torch.empty(R, -(-K // per), dtype=torch.int32, device=dev)
    qz = torch.empty(R, -(-G // per), dtype=torch.int32, device=dev)
    sc = torch.empty(R, G, dtype=torch.float16, device=dev)
    import contextlib
    # overrides run on the diagnostics build (_hip.tuning); the defaults on the shipped library
    ctx = _hip.tuning(no_rowgroup=int(generic), **(tun or {})) if (generic or tun) else contextlib.nullcontext()
    ctx.__enter__()
    stage = {}
    if args.search or generic or not _hip.packs_directly(DT[name], R, K, gs):
        stage = dict(tensor_q=torch.empty(R * K, dtype=torch.int32, device=dev),
                     zeros=torch.empty(R, G, dtype=torch.int32, device=dev))

    def run():
        if args.search:
            _hip.quantize_search(x, R, K, gs, args.bits, False, 20, args.search, qweight=qw, qzeros=qz, scales=sc,
                                 **stage)
        else:
            _hip.quantize_groups(x, R, K, gs, args.bits, False, qweight=qw, qzeros=qz, scales=sc, **stage)
    for _ in range(3):
        run()
    settle(args, _hip, dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(args.iters):
        run()
    b.record()
    torch.cuda.synchronize()
    ctx.__exit__(None, None, None)
    us = a.elapsed_time(b) / args.iters * 1e3
    # the outputs' bytes: equal across A/B builds = same results
    h = hashlib.sha256()
    for t in (qw, qz, sc, *stage.values()):
        h.update(t.cpu().numpy().tobytes())
    nbytes = x.numel() * x.element_size()
    algo = nbytes + sum(t.numel() * t.element_size() for t in (qw, qz, sc))
    kernel = ("generic+pack" if stage and not args.search else "search" if args.search else
              "generic" if generic or name == "f64" or gs > (256 if name == "f32" else 512) else
              "streaming" if _hip.ragged_eligible(DT[name], R, K, gs) else "row-segment")
    print(json.dumps({"dtype": name, "shape": [R, K], "group_size": gs, "bits": args.bits, "kernel": kernel, "tuning": tun or {},
                      "lib": os.path.basename(args.lib) if args.lib else "libawq_hip.so",
                      "search": args.search, "us": round(us, 1), "input_GBs": round(nbytes / us / 1e3, 1),
                      "algorithmic_GBs": round(algo / us / 1e3, 1), "frac_8TBs": round(algo / us / 1e3 / 8000, 3),
                      "out_sha": h.hexdigest()[:16], "settle_ms": args.settle_ms}),
          flush=True)
    if args.dequant:
        out = torch.empty(R, K, dtype=torch.float32, device=dev)

        def dq():
            _hip.dequantize_packed(qw, qz, sc, R, K, gs, args.bits, False, out)
        variants = tuple(int(v) for v in args.dq_variants.split(",")) if args.dq_ab else (0,)
        ref = None
        for rnd in range(3 if args.dq_ab else 1):
            for v in variants:
                with (_hip.tuning(dq_words_v1=v) if v else contextlib.nullcontext()):
                    for _ in range(3):
                        dq()
                    settle(args, _hip, dev)
                    a.record()
                    for _ in range(args.iters):
                        dq()
                    b.record()
                    torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                same = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
                us = a.elapsed_time(b) / args.iters * 1e3
                algo = out.numel() * 4 + sum(t.numel() * t.element_size() for t in (qw, qz, sc))
                print(json.dumps({"op": "dequantize_packed", "lib": os.path.basename(args.lib) if args.lib else "libawq_hip.so", "kernel": ["default", "words_v1", "words_v2_xcd", "words_v2", "quads", "quads_xcd", "batch4", "batch8", "batch4_run4", "batch8_run2"][v], "round": rnd,
                                  "shape": [R, K], "group_size": gs, "bits": args.bits, "same_bits": same,
                                  "us": round(us, 1), "algorithmic_GBs": round(algo / us / 1e3, 1),
                                  "frac_8TBs": round(algo / us / 1e3 / 8000, 3)}), flush=True)


if __name__ == "__main__":
    main()
