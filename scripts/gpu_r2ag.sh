#!/bin/bash
# round 2: row-segment default plan with whole-row two-wave tiles: parity (defaults and
# forced one-wave), then defaults vs AWQ_RG_WAVES=1 (the one-wave cost model) per shape
set -u
OUT=gpurun_out/r2ag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rowgroup.py tests/test_gpu_group_sizes.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
AWQ_RG_WAVES=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_rowgroup.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_w1.log 2>&1 || exit $?
for M in default w1; do
  if [ $M = w1 ]; then export AWQ_RG_WAVES=1; else unset AWQ_RG_WAVES; fi
  timeout -k 10 300 python scripts/generic_bench.py --shape "14336,4096;4096,14336;4096,2048;8192,3000" --dtypes bf16,f16,f32 --group-sizes 100,96,200,300,500,60 > $OUT/$M.log 2>&1 || exit $?
done
echo done
