#!/bin/bash
# round 2: row-segment two-wave tiles inside long rows (G > 64): groups-per-tile sweep at
# 2 waves vs the one-wave default
set -u
OUT=gpurun_out/r2ai
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python scripts/generic_bench.py --shape "4096,14336;14336,4096" --dtypes bf16 --group-sizes 100,96,60,48,40 > $OUT/default.log 2>&1 || exit $?
for G in 32 40 48 56 64; do
  AWQ_RG_WAVES=2 AWQ_RG_GPT=$G timeout -k 10 120 python scripts/generic_bench.py --shape "4096,14336;14336,4096" --dtypes bf16 --group-sizes 100,96,60,48,40 > $OUT/w2_gpt$G.log 2>&1 || exit $?
done
timeout -k 10 120 python scripts/generic_bench.py --shape "4096,14336;14336,4096" --dtypes bf16 --group-sizes 100,96,60,48,40 > $OUT/default_again.log 2>&1 || exit $?
echo done
