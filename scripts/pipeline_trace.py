#!/usr/bin/env python3
"""Per-batch table of a traced CLI run (scripts/cli_first_run.py --trace / cli_bench.py): for
each batch the read window, the H2D / kernel / D2H windows on the event clock and the host
time spent in the H2D / D2H calls, plus the totals that say which leg bounds the pipeline.

  python scripts/pipeline_trace.py <log> [--run N] [--rows]
"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--run", type=int, default=0, help="which traced result line (0 = first)")
    ap.add_argument("--rows", action="store_true", help="print every batch")
    a = ap.parse_args()
    runs = []
    for ln in open(a.log):
        if not ln.startswith("{"):
            continue
        d = json.loads(ln)
        ph = d.get("phases") or {}
        st = [v for k, v in ph.items() if k.startswith("stream_") and isinstance(v, dict) and v.get("trace")]
        if st:
            runs.append((d, ph, st[0]))
    d, ph, st = runs[a.run]
    tr = st["trace"]
    h2d = [b["h2d_done"] - max(b["h2d_enq"], (tr[i - 1]["h2d_done"] if i else 0)) for i, b in enumerate(tr)]
    print(json.dumps({k: d.get(k) for k in ("workload", "format", "run", "main_s", "process_wall_s")}))
    print(json.dumps({k: v for k, v in st.items() if k != "trace"}))
    print(json.dumps({k: v for k, v in ph.items() if not k.startswith("stream_")}))
    nb = len(tr)
    first = tr[0]
    last = tr[-1]
    print(f"batches {nb}: first read starts {first['read_first']:.4f}, first H2D enqueued {first['h2d_enq']:.4f}, "
          f"first kernels enqueued {first['kern_enq']:.4f} (launch {first['ragged_launch']:.4f}), "
          f"last D2H done {last['d2h_done']:.4f}")
    print(f"sum of H2D windows {sum(h2d):.4f} s; reads: last read ends {max(b['read_last'] for b in tr):.4f}")
    if a.rows:
        for i, b in enumerate(tr):
            print(f"{i:3d} read {b['read_first']:.4f}-{b['read_last']:.4f}  h2d {b['h2d_enq']:.4f}->{b['h2d_done']:.4f} "
                  f"({h2d[i] * 1e3:5.1f} ms)  kern {b['kern_enq']:.4f}->{b['kern_done']:.4f}  "
                  f"d2h {b['d2h_enq']:.4f}->{b['d2h_done']:.4f}  calls h2d {b['h2d_call'] * 1e3:.2f} d2h {b['d2h_call'] * 1e3:.2f} ms")


if __name__ == "__main__":
    main()
