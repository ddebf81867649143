#!/bin/bash
# round 2: full GPU suite + smoke + default bench after the row-segment / act-search changes;
# row-segment defaults per group size with rocprof kernel stats
set -u
OUT=gpurun_out/r2aa
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16,f16,f32 --group-sizes 100,48,96,60,200,300 > $OUT/gs_default.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_rg -o rg --output-format csv -- python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16 --group-sizes 100 > $OUT/prof_rg.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
echo done
