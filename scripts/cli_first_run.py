#!/usr/bin/env python3
"""The CLI as users run it: ONE fresh process per invocation (reference main.py:515-676 runs
once per process), on a synthetic multi-file checkpoint with a BASELINE config's exact
shapes, page cache warm.  Per run, the phases of the child process separately:

  interp_s         process start -> first line of the driver (python interpreter)
  warmup_start_s   _early.start: HIP's first-use work begins on a native thread (it then
                   overlaps the import of torch; TIMINGS warmup_s = its duration, the
                   pipeline's prepare_s = how long the pipeline still waited for it)
  torch_s          import torch
  import_s         import awq_quantizer.main (+ libawq_hip.so load)
  main_s           awq_quantizer.main.main(argv): torch's CUDA init (TIMINGS device_s),
                   index, pipeline, chunk files, metadata, with the CLI's own phase times
                   (TIMINGS) beside it

plus the plain `python -m awq_quantizer.main ...` command timed whole by the parent.

  python scripts/cli_first_run.py --workload llama3-8b --shards 4 --formats packed --runs 2
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(argv_json, t_spawn, trace="0", opts="{}"):
    # the order of `python -m awq_quantizer.main`: the device warm-up starts (main.py's
    # module top, _early.py), torch is imported, main() runs — torch's CUDA init and the
    # wait for the warm-up fall inside main() and are reported from its TIMINGS
    t0 = time.time()
    sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
    argv = json.loads(argv_json)
    if os.environ.get("CLI_FIRST_RUN_NO_EARLY") != "1":      # (A/B: the warm-up left to the pipeline)
        from awq_quantizer import _early
        _early.start(argv)
    t1 = time.time()
    import torch  # noqa: F401
    t2 = time.time()
    from awq_quantizer import main as cli
    from awq_quantizer import _hip
    _hip.load_library()
    t3 = time.time()
    if trace == "1":
        cli.STREAM_OPTS["trace"] = 1
    cli.STREAM_OPTS.update(json.loads(opts))
    rc = cli.main(argv)
    t4 = time.time()
    ph = {k: v for k, v in cli.TIMINGS.items()}
    print("RESULT " + json.dumps({"rc": rc, "interp_s": round(t0 - t_spawn, 3), "warmup_start_s": round(t1 - t0, 3),
                                  "torch_s": round(t2 - t1, 3), "import_s": round(t3 - t2, 3),
                                  "main_s": round(t4 - t3, 3), "phases": ph}, default=str), flush=True)


def warm(model):
    for f in sorted(os.listdir(model)):
        with open(os.path.join(model, f), "rb") as fh:
            while fh.read(1 << 26):
                pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="opt-350m")
    ap.add_argument("--shards", type=int, default=3)
    ap.add_argument("--formats", default="packed,reference")
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--trace", action="store_true", help="per-batch pipeline trace in the phases")
    ap.add_argument("--opts", default="{}", help="JSON merged into main.STREAM_OPTS (A/B of pipeline sizes)")
    ap.add_argument("--no-early", action="store_true", help="do not start the warm-up before import torch (A/B)")
    ap.add_argument("--child", nargs=4)
    a = ap.parse_args()
    if a.child:
        child(a.child[0], float(a.child[1]), a.child[2], a.child[3])
        return
    sys.path[:0] = [ROOT, os.path.join(ROOT, "scripts")]
    import cli_bench
    work = a.workdir or tempfile.mkdtemp(prefix="awq_first_")
    model = os.path.join(work, f"model_{a.workload}")
    os.makedirs(model, exist_ok=True)
    t = time.time()
    nbytes = cli_bench.build_model(model, a.workload, a.shards)
    print(json.dumps({"workload": a.workload, "files": a.shards, "input_GB": round(nbytes / 1e9, 3),
                      "build_s": round(time.time() - t, 1)}), flush=True)
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "awq-converter_amd"), ROOT]),
               CLI_FIRST_RUN_NO_EARLY="1" if a.no_early else "0")
    for fmt in a.formats.split(","):
        for r in range(a.runs):
            warm(model)
            out = os.path.join(work, f"out_{fmt}_{r}")
            argv = ["--model_id", model, "--output_dir", out, "--log_level", "WARNING", "--output_format", fmt]
            t_spawn = time.time()
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", json.dumps(argv), repr(t_spawn),
                                "1" if a.trace else "0", a.opts],
                               capture_output=True, text=True, timeout=600, env=env)
            wall = time.time() - t_spawn
            res = [ln[7:] for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
            if p.returncode or not res:
                print(json.dumps({"format": fmt, "run": r, "rc": p.returncode, "err": p.stderr[-1500:]}), flush=True)
                sys.exit(1)
            d = json.loads(res[0])
            ob = sum(os.path.getsize(os.path.join(out, f)) for f in os.listdir(out))
            d.update({"workload": a.workload, "format": fmt, "run": r, "kind": "fresh process, page cache warm",
                      "opts": json.loads(a.opts), "early_warmup": not a.no_early,
                      "process_wall_s": round(wall, 3), "input_GB": round(nbytes / 1e9, 3),
                      "output_GB": round(ob / 1e9, 3), "main_input_GBs": round(nbytes / d["main_s"] / 1e9, 2)})
            print(json.dumps(d), flush=True)
            shutil.rmtree(out, ignore_errors=True)
        # the command itself, timed whole
        warm(model)
        out = os.path.join(work, f"out_{fmt}_cmd")
        t = time.time()
        p = subprocess.run([sys.executable, "-m", "awq_quantizer.main", "--model_id", model, "--output_dir", out,
                            "--log_level", "WARNING", "--output_format", fmt], capture_output=True, text=True,
                           timeout=600, env=env)
        print(json.dumps({"workload": a.workload, "format": fmt, "command": "python -m awq_quantizer.main",
                          "rc": p.returncode, "wall_s": round(time.time() - t, 3)}), flush=True)
        shutil.rmtree(out, ignore_errors=True)
    if a.workdir is None:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
