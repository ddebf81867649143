#!/bin/bash
# round 2: strided span (fp64 at other group sizes, groups > 512, forced generic) with every
# group's lane-local min/max first (4 loads in flight per lane), the groups' butterflies
# interleaved and NaN by ballot — parity, A/B against the previous build (variants/dpp), then
# the full GPU suite, smoke and the default bench line on the final library.
set -u
OUT=gpurun_out/r2aq
mkdir -p $OUT
export TMPDIR=/tmp
PREV=awq-converter_amd/awq_quantizer/_lib/variants/dpp/libawq_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_generic_span.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_span.log 2>&1 || exit $?
GB="--shape 14336,4096;4096,14336 --dtypes f64 --group-sizes 100,96,1024"
GB2="--shape 14336,4096 --dtypes bf16,f32 --group-sizes 1024,2048"
for R in 1 2; do
  timeout -k 10 120 python scripts/generic_bench.py $GB > $OUT/new_f64_$R.log 2>&1 || exit $?
  AWQ_HIP_LIB=$PREV timeout -k 10 120 python scripts/generic_bench.py $GB > $OUT/prev_f64_$R.log 2>&1 || exit $?
done
timeout -k 10 120 python scripts/generic_bench.py $GB2 > $OUT/new_large.log 2>&1 || exit $?
AWQ_HIP_LIB=$PREV timeout -k 10 120 python scripts/generic_bench.py $GB2 > $OUT/prev_large.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
echo done
