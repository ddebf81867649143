#!/bin/bash
# round 2: row-segment tiles shared by 2 waves (128-thread workgroups): parity at 1 and 2
# waves per tile, then a groups-per-tile x waves-per-tile sweep
set -u
OUT=gpurun_out/r2af
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rowgroup.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_w1.log 2>&1 || exit $?
AWQ_RG_WAVES=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_rowgroup.py tests/test_gpu_group_sizes.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_w2.log 2>&1 || exit $?
for W in 1 2; do
  for G in 8 16 24 32 48 64; do
    AWQ_RG_WAVES=$W AWQ_RG_GPT=$G timeout -k 10 120 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16 --group-sizes 100,48,96,60,200,40,24 > $OUT/w${W}_gpt$G.log 2>&1 || exit $?
  done
done
echo done
