#!/bin/bash
# The one GPU-box launcher: runs named steps in order, each under its own time limit, output
# to gpurun_out/<tag>/<name>.log; the first failing step ends the call (a GPU fault, abort or
# time limit must not be followed by more GPU work).
#
#   bash scripts/gpu_run.sh <tag> <step> [<step> ...]
#
# step = name:seconds:command   (the command is run by bash; ':' may appear in it)
# shorthands:
#   pytest[=<pytest args>]   full GPU suite (default) or a selection, 120 s per test
#   smoke                    __graft_entry__.smoke()
#   bench[=<bench.py args>]  bench.py line
#   rocprof_bench            rocprofv3 --kernel-trace --stats of the default bench (20 launches)
#   pmc=<regex>=<counter>=<python args>   one rocprofv3 --pmc pass (kernel-trace only)
# e.g.  gpurun -- 'bash scripts/gpu_run.sh r3a pytest smoke bench rocprof_bench'
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  case "$step" in
    pytest) name=pytest_gpu; secs=1500
            cmd="python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" ;;
    pytest=*) name=pytest_$n; secs=900
            cmd="python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${step#pytest=}" ;;
    smoke) name=smoke; secs=300; cmd="python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" ;;
    bench) name=bench; secs=600; cmd="python bench.py" ;;
    bench=*) name=bench_$n; secs=600; cmd="python bench.py ${step#bench=}" ;;
    rocprof_bench) name=rocprof_bench; secs=600
            cmd="rocprofv3 --kernel-trace --stats --kernel-include-regex awq_fast_kernel -d $OUT/trace -o bench --output-format csv -- python bench.py --steps 20 --no-cpu-baseline" ;;
    pmc=*) IFS='=' read -r _ rx ctr pyargs <<< "$step"
           name=pmc_${n}_$ctr; secs=120
           cmd="timeout -s KILL 100 rocprofv3 --kernel-include-regex '$rx' --pmc $ctr --output-format csv -d $OUT/pmc_$n -o p -- python $pyargs" ;;
    *:*:*) name=${step%%:*}; rest=${step#*:}; secs=${rest%%:*}; cmd=${rest#*:} ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "=== [$n] $name ($secs s): $cmd" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "=== [$n] $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -4 "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "step $name failed (rc=$rc): stopping"; exit $rc; }
done
echo done
