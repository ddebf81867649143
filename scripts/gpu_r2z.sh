#!/bin/bash
# round 2: row-segment groups per tile, any multiple of 8 (override sweep), parity first; per-tile lanes per group; XCD-contiguous tiles
set -u
OUT=gpurun_out/r2z3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rowgroup.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
for G in 24 40 48; do
  AWQ_RG_GPT=$G timeout -k 10 300 python -u -m pytest tests/test_gpu_rowgroup.py -x -q --timeout 120 --timeout-method thread -k "bfloat16 and not special" > $OUT/pytest_gpt$G.log 2>&1 || exit $?
done
for G in 8 16 24 32 40 48 56 64; do
  AWQ_RG_GPT=$G timeout -k 10 120 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16 --group-sizes 100,48,96,60,200,40,24 > $OUT/gpt$G.log 2>&1 || exit $?
done
echo done
