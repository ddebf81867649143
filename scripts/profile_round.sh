#!/bin/bash
# rocprofv3 evidence for the bench line (run on the GPU box from the repo root):
#   1. kernel trace + stats of `bench.py` (default workload)  -> gpurun_out/<tag>/trace
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate --pmc runs, kernel-trace only)
#   4. pmc_traffic.py -> profiles/pmc_traffic.json (bench.py reads it for roofline.traffic)
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---no-cpu-baseline}            # bench defaults: 500 warmup + 1000 timed launches
PMC_ARGS=${PMC_ARGS:---steps 20 --warmup 5 --no-cpu-baseline --no-copy-ceiling}   # counters: per-dispatch, keep it short
run() { local name=$1; shift; echo "=== $name"; timeout -k 10 400 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -2 "$OUT/$name.log"; [ $rc -eq 0 ] || exit $rc; }
run trace rocprofv3 --kernel-trace --stats --kernel-include-regex 'awq_fast_kernel' -d "$OUT/trace" -o bench --output-format csv -- python bench.py $ARGS
run fetch rocprofv3 --kernel-include-regex 'awq_fast_kernel' --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o bench -- python bench.py $PMC_ARGS
run write rocprofv3 --kernel-include-regex 'awq_fast_kernel' --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o bench -- python bench.py $PMC_ARGS
ALGO=$(grep '^{"metric"' "$OUT/trace.log" | tail -1 | python -c "import json,sys;print(json.loads(sys.stdin.read())['roofline']['algorithmic_bytes_per_launch'])")
python scripts/pmc_traffic.py --fetch "$OUT/fetch" --write "$OUT/write" --key "${TRAFFIC_KEY:-opt-125m.b4.asym.packed}" --algo-bytes "$ALGO" \
  --out "$OUT/pmc_traffic.json"
python scripts/trace_window.py "$OUT/trace/bench_kernel_trace.csv" --steps "${WINDOW_STEPS:-1000}" > "$OUT/trace_window.json"
cat "$OUT/trace_window.json"
find "$OUT" -name '*counter_collection.csv' -size +2M -delete
echo done
