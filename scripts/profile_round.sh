#!/bin/bash
# rocprofv3 evidence for the bench line (run on the GPU box from the repo root):
#   1. kernel trace + stats of `bench.py` (default workload: Llama-3-70B) -> gpurun_out/<tag>/trace
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate --pmc runs, kernel-trace only)
#   4. pmc_traffic.py -> gpurun_out/<tag>/pmc_traffic.json (copied into profiles/roundN/
#      pmc_traffic.json, which bench.py reads for roofline.traffic, labelled as recorded)
set -u
TAG=${1:-round2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---no-cpu-baseline}
STEPS=${STEPS:-20}
PMC_ARGS=${PMC_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling ${WL_ARGS:-}}   # counters: per dispatch
run() { local name=$1; shift; echo "=== $name"; timeout -k 10 ${STEP_TIMEOUT:-300} "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -2 "$OUT/$name.log"; [ $rc -eq 0 ] || exit $rc; }
run trace rocprofv3 --kernel-trace --stats --kernel-include-regex 'awq_fast_kernel' -d "$OUT/trace" -o bench --output-format csv -- python bench.py --steps $STEPS $ARGS ${WL_ARGS:-}
run fetch rocprofv3 --kernel-include-regex 'awq_fast_kernel' --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o bench -- python bench.py $PMC_ARGS
run write rocprofv3 --kernel-include-regex 'awq_fast_kernel' --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o bench -- python bench.py $PMC_ARGS
ALGO=$(grep '^{"metric"' "$OUT/trace.log" | tail -1 | python -c "import json,sys;print(json.loads(sys.stdin.read())['roofline']['algorithmic_bytes_per_launch'])")
python scripts/pmc_traffic.py --fetch "$OUT/fetch" --write "$OUT/write" --key "${TRAFFIC_KEY:-llama3-70b.b4.asym.packed}" \
  --algo-bytes "$ALGO" --commit "${COMMIT:-unknown}" --date "$(date -u +%Y-%m-%d)" --out "${TRAFFIC_OUT:-$OUT/pmc_traffic.json}"
python scripts/trace_window.py "$OUT/trace/bench_kernel_trace.csv" --steps "$STEPS" > "$OUT/trace_window.json"
cat "$OUT/trace_window.json"
find "$OUT" -name '*counter_collection.csv' -size +2M -delete
echo done
