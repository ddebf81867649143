#!/bin/bash
# One GPU-box session: smoke -> parity tests -> bench -> rocprofv3 kernel trace.
# Each GPU step has its own time limit; a fault/abort/timeout stops the script.
# Usage (from the repo root on the box): bash scripts/gpu_round.sh [tag]
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() {  # exit codes that mean the GPU step crashed/hung: stop everything
  case $1 in 124|137|134|139|-6|-11) return 0;; *) return 1;; esac
}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name; stopping"; exit $rc; fi
  return $rc
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
run bench 600 python bench.py
for WL in ${BENCH_EXTRA:-}; do
  run bench_$WL 900 python bench.py --workload $WL --steps 10 --warmup 3 --no-cpu-baseline
done
if [ "${PROFILE:-1}" = 1 ]; then
  COMMIT=${COMMIT:-unknown} bash scripts/profile_round.sh "$TAG/prof" || exit 1
fi
echo done
