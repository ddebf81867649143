#!/bin/bash
# round 2: fp64 register-resident span with DPP for the in-row reduction levels and the pack OR (was: LDS
# bpermute shuffles) — parity, then A/B against the previous register-resident build (variants/reg2),
# interleaved; rocprof stats.
set -u
OUT=gpurun_out/r2ap
mkdir -p $OUT
export TMPDIR=/tmp
REG2=awq-converter_amd/awq_quantizer/_lib/variants/reg2/libawq_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_generic_span.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_span.log 2>&1 || exit $?
GB="--shape 14336,4096;4096,14336 --dtypes f64 --group-sizes 128,64 --bits 4"
GB8="--shape 14336,4096 --dtypes f64 --group-sizes 128 --bits 8"
for R in 1 2; do
  timeout -k 10 120 python scripts/generic_bench.py $GB > $OUT/new_f64_$R.log 2>&1 || exit $?
  AWQ_HIP_LIB=$REG2 timeout -k 10 120 python scripts/generic_bench.py $GB > $OUT/reg2_f64_$R.log 2>&1 || exit $?
done
timeout -k 10 120 python scripts/generic_bench.py $GB8 > $OUT/new_f64_b8.log 2>&1 || exit $?
AWQ_HIP_LIB=$REG2 timeout -k 10 120 python scripts/generic_bench.py $GB8 > $OUT/reg2_f64_b8.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o gen --output-format csv -- python scripts/generic_bench.py --shape 14336,4096 --dtypes f64 --group-sizes 128 > $OUT/prof.log 2>&1 || exit $?
echo done
