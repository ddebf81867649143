#!/bin/bash
# round 2: row-segment pass 2 with a float induction for the group index (A/B vs the
# previous library built from the same sources at HEAD, interleaved in one process each)
set -u
OUT=gpurun_out/r2al
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rowgroup.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
for R in 1 2; do
  timeout -k 10 120 python scripts/generic_bench.py --shape "14336,4096;4096,14336" --dtypes bf16,f16 --group-sizes 100,96,60,200 > $OUT/new_$R.log 2>&1 || exit $?
  AWQ_HIP_LIB=awq-converter_amd/awq_quantizer/_lib/variants/libawq_hip_prev.so timeout -k 10 120 python scripts/generic_bench.py --shape "14336,4096;4096,14336" --dtypes bf16,f16 --group-sizes 100,96,60,200 > $OUT/prev_$R.log 2>&1 || exit $?
done
echo done
