#!/bin/bash
# round 2: full GPU suite + smoke + default bench with the two-wave whole-row default; rocprof
# kernel stats of the bf16 gs-100 row-segment launch
set -u
OUT=gpurun_out/r2aj
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_rg -o rg --output-format csv -- python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16 --group-sizes 100 > $OUT/prof_rg.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
echo done
