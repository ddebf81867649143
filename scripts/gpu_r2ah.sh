#!/bin/bash
# round 2: row-segment whole-row tiles at 2 vs 4 waves per tile (tuning overrides)
set -u
OUT=gpurun_out/r2ah
mkdir -p $OUT
export TMPDIR=/tmp
AWQ_RG_WAVES=4 AWQ_RG_GPT=48 timeout -k 10 300 python -u -m pytest tests/test_gpu_rowgroup.py -x -q --timeout 120 --timeout-method thread -k "not override" > $OUT/pytest_w4.log 2>&1 || exit $?
for W in 2 4; do
  AWQ_RG_WAVES=$W AWQ_RG_GPT=48 timeout -k 10 120 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16,f16 --group-sizes 100,96 > $OUT/w${W}_gpt48.log 2>&1 || exit $?
  AWQ_RG_WAVES=$W AWQ_RG_GPT=24 timeout -k 10 120 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16,f16 --group-sizes 200 > $OUT/w${W}_gpt24.log 2>&1 || exit $?
  AWQ_RG_WAVES=$W AWQ_RG_GPT=16 timeout -k 10 120 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16 --group-sizes 300,500 > $OUT/w${W}_gpt16.log 2>&1 || exit $?
done
timeout -k 10 120 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16,f16 --group-sizes 100,96,200,300,500 > $OUT/default.log 2>&1 || exit $?
echo done
