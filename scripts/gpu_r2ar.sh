#!/bin/bash
# round 2, final tree: full GPU suite, smoke, default bench line, and the rocprof kernel-trace
# stats of the default bench (Llama-3-70B set) for the committed profiles.
set -u
OUT=gpurun_out/r2ar
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --kernel-include-regex 'awq_fast_kernel' -d $OUT/trace -o bench --output-format csv -- python bench.py --steps 20 --no-cpu-baseline > $OUT/bench_under_rocprof.log 2>&1 || exit $?
echo done
