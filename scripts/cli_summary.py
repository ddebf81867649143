#!/usr/bin/env python3
"""Compact table of scripts/cli_first_run.py logs: per fresh-process run the child's phases
(interpreter, warm-up start, import torch, import of the CLI, main()), main()'s own phase
times (setup, pipeline, the pipeline's wait for the device warm-up, the writer's close
wait) and the plain `python -m awq_quantizer.main` wall, as one JSON line each.

  python scripts/cli_summary.py <log> [<log> ...]
"""
import json
import sys


def main():
    for path in sys.argv[1:]:
        for ln in open(path):
            if not ln.startswith("{"):
                continue
            d = json.loads(ln)
            if "command" in d:
                print(json.dumps({"log": path, "workload": d["workload"], "format": d["format"], "command": d["command"],
                                  "wall_s": d["wall_s"]}))
                continue
            if "main_s" not in d:
                continue
            ph = d.get("phases") or {}
            st = next((v for k, v in ph.items() if k.startswith("stream_") and isinstance(v, dict)), {})
            wr = ph.get("writer") or {}
            gb = d["input_GB"]
            print(json.dumps({
                "log": path, "workload": d["workload"], "format": d["format"], "run": d["run"],
                "early_warmup": d.get("early_warmup", d.get("warmup_start_s", 0) > 0), "opts": d.get("opts", {}),
                "process_wall_s": d["process_wall_s"], "interp_s": d["interp_s"], "torch_s": d["torch_s"],
                "main_s": d["main_s"], "main_GBs": round(gb / d["main_s"], 1),
                "setup_s": st.get("setup_s"), "pipeline_s": st.get("pipeline_s"),
                "pipeline_GBs": round(gb / st["pipeline_s"], 1) if st.get("pipeline_s") else None,
                "warmup_s": st.get("warmup_s"), "pipeline_wait_warmup_s": st.get("prepare_s"),
                "host_ring_MB": st.get("host_ring_MB"), "wait_release_s": st.get("submit_wait_release_s"),
                "writer_close_wait_s": wr.get("close_wait_s"), "input_GB": gb, "output_GB": d.get("output_GB")}))


if __name__ == "__main__":
    main()
