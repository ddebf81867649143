#!/usr/bin/env python3
"""End-to-end CLI throughput (safetensors on disk -> quantized chunks on disk), the
reference's own use case (main.py).  Builds a synthetic model directory with a tensor
set's exact shapes (bench.py manifests), runs awq_quantizer.main.main() on it and reports
wall time and GB/s of bf16 input, plus the time split the CLI logs.

  python scripts/cli_bench.py --workload opt-125m --format packed
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

import bench  # noqa: E402


def build_model(path, workload, shards):
    shapes = bench.shapes_of(workload)
    if os.path.exists(os.path.join(path, "complete")):    # reuse a model built by an earlier run (--workdir)
        return sum(int(torch.Size(s).numel()) * 2 for s in shapes)
    # generated on the GPU when there is one (a 16 GB checkpoint in seconds, not minutes), with
    # a progress line per shard (a silent multi-minute build looks hung to the GPU runner)
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    g = torch.Generator(device=dev).manual_seed(0)
    names = [f"model.layers.{i // 8}.t{i}.weight" for i in range(len(shapes))]
    per = -(-len(shapes) // shards)
    nbytes = 0
    for sh in range(shards):
        part = {}
        for n, s in list(zip(names, shapes))[sh * per:(sh + 1) * per]:
            part[n] = (torch.randn(*s, generator=g, device=dev) * 0.02).to(torch.bfloat16).cpu()
            nbytes += part[n].numel() * 2
        if part:
            save_file(part, os.path.join(path, f"model-{sh:05d}-of-{shards:05d}.safetensors"))
            print(f"build_model: shard {sh + 1}/{shards} written ({nbytes / 1e9:.1f} GB so far)", flush=True)
    open(os.path.join(path, "complete"), "w").close()
    return nbytes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="opt-125m", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--format", default="packed", choices=["packed", "reference"])
    ap.add_argument("--shards", type=int, default=2)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--repeat", type=int, default=2)
    args = ap.parse_args()
    from awq_quantizer import main as cli_mod
    cli = cli_mod.main
    work = args.workdir or tempfile.mkdtemp(prefix="awq_cli_")
    model = os.path.join(work, "model")
    os.makedirs(model, exist_ok=True)
    t0 = time.time()
    nbytes = build_model(model, args.workload, args.shards)
    build_s = time.time() - t0
    for r in range(args.repeat):
        out = os.path.join(work, f"out{r}")
        t0 = time.time()
        rc = cli(["--model_id", model, "--output_dir", out, "--log_level", "WARNING", "--output_format", args.format])
        wall = time.time() - t0
        assert rc == 0
        out_bytes = sum(os.path.getsize(os.path.join(out, f)) for f in os.listdir(out))
        print(json.dumps({"workload": args.workload, "format": args.format, "run": r, "input_GB": round(nbytes / 1e9, 3),
                          "output_GB": round(out_bytes / 1e9, 3), "wall_s": round(wall, 3),
                          "input_GBs": round(nbytes / wall / 1e9, 3), "model_build_s": round(build_s, 1),
                          "serial_save": os.environ.get("AWQ_CLI_SERIAL_SAVE", "0") == "1",
                          "phases_s": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in cli_mod.TIMINGS.items()}}), flush=True)
        shutil.rmtree(out, ignore_errors=True)
    if args.workdir is None:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
