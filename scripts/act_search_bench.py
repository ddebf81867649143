#!/usr/bin/env python3
"""Timing of the activation-aware scale search (scale_method="awq", include/awq_hip.h
awq_act_*) on one transformer block's layer groups at Llama-3-8B shapes (synthetic bf16
weights, synthetic calibration activations).  Per step: HIP-event time of each launch
sequence, candidate-elements per second for the loss kernel.

  python scripts/act_search_bench.py --tokens 512 --grid 20
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402

GROUPS = {   # layer group -> (rows of each linear sharing the input, in_features)
    "qkv": ([4096, 1024, 1024], 4096),
    "o": ([4096], 4096),
    "gate_up": ([14336, 14336], 4096),
    "down": ([4096], 14336),
}


def timed(fn, iters):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        out = fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=512)
    ap.add_argument("--grid", type=int, default=20)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--groups", default=",".join(GROUPS))
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16"])
    ap.add_argument("--lib", default="", help="load this in-tree build instead of _lib/libawq_hip.so (A/B of builds)")
    args = ap.parse_args()
    from awq_quantizer import _hip
    if args.lib:
        _hip.load_library(args.lib)
    from awq_quantizer.quantization import AWQQuantizer
    dev = torch.device("cuda", 0)
    _hip.require_device(dev)
    q = AWQQuantizer(bits=4, group_size=128, symmetric=False, scale_method="awq", search_grid=args.grid,
                     device="cuda", logger_level="ERROR")
    for gname in args.groups.split(","):
        rows, K = GROUPS[gname]
        g = torch.Generator(device=dev).manual_seed(0)
        dt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
        ws = [(torch.randn(r, K, device=dev, generator=g) * 0.02).to(dt) for r in rows]
        x = (torch.randn(args.tokens, K, device=dev, generator=g) * 2).to(dt)
        elems = sum(r * K for r in rows)
        t_stats, (xm, xs) = timed(lambda: _hip.act_stats(x), args.iters)
        t_wmean, wm = timed(lambda: _hip.weight_mean(ws, 128), args.iters)
        t_table, table = timed(lambda: _hip.act_scale_table(xm, wm, args.grid), args.iters)
        t_table1, _ = timed(lambda: _hip.act_scale_table(xm, wm, args.grid, workspace=False), args.iters)
        t_loss, part = timed(lambda: _hip.act_search_losses(ws, xs, table, 128, 4, False), args.iters)
        t_sel, (losses, best, s) = timed(lambda: _hip.act_search_select(part, table), args.iters)
        t_apply, _ = timed(lambda: [q.quantize_packed(_hip.apply_input_scale(w, s)) for w in ws], args.iters)

        def one_pass():
            for w in ws:
                r = q._packed_outputs(w)
                _hip.quantize_groups_scaled(w, s, 128, 4, False, qweight=r["qweight"], qzeros=r["qzeros"],
                                            scales=r["scales"])
        t_scaled, _ = timed(one_pass, args.iters)
        t_all, _ = timed(lambda: q.quantize_layer_group({str(i): w for i, w in enumerate(ws)}, x), args.iters)
        print(json.dumps({"group": gname, "dtype": args.dtype, "rows": rows, "K": K, "tokens": args.tokens, "grid": args.grid,
                          "weights_MB": round(elems * 2 / 1e6, 1), "us": {
                              "act_stats": round(t_stats, 1), "weight_mean": round(t_wmean, 1),
                              "scale_table": round(t_table, 1), "scale_table_no_ws": round(t_table1, 1),
                              "losses": round(t_loss, 1),
                              "select": round(t_sel, 1), "apply+quantize": round(t_apply, 1),
                              "scaled_quantize_one_pass": round(t_scaled, 1),
                              "quantize_layer_group": round(t_all, 1)},
                          "loss_Gcand_elem_per_s": round(elems * args.grid / t_loss / 1e3, 1),
                          "loss_weight_GBs_per_candidate": round(elems * 2 * args.grid / t_loss / 1e3, 1),
                          "best": int(best.item()),
                          # the loss partials' bytes: equal across A/B builds = same results
                          "part_sha": hashlib.sha256(part.cpu().numpy().tobytes()).hexdigest()[:16],
                          "lib": os.path.basename(args.lib) if args.lib else "libawq_hip.so"}), flush=True)


if __name__ == "__main__":
    main()
