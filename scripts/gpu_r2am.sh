#!/bin/bash
# round 2 (re-entry): generic kernel rewritten as one wave per qzeros-word span with in-kernel
# packing (fp64, groups > 512).  New parity tests first, then an A/B against the previous
# library (generic kernel + int32 staging + pack passes), then the full GPU suite, smoke and
# the default bench line; rocprof stats of the fp64 launch.  Word-per-thread packed dequantize
# A/B in the same call.
set -u
OUT=gpurun_out/r2am
mkdir -p $OUT
export TMPDIR=/tmp
PREV=awq-converter_amd/awq_quantizer/_lib/variants/prev/libawq_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_generic_span.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_span.log 2>&1 || exit $?
GB="--shape 14336,4096;4096,14336 --dtypes f64 --group-sizes 128,100,1024"
GB2="--shape 14336,4096 --dtypes bf16 --group-sizes 1024,2048"
GD="--shape 14336,4096;128256,4096 --dtypes bf16 --group-sizes 128,32 --dequant"
for R in 1 2; do
  timeout -k 10 120 python scripts/generic_bench.py $GB > $OUT/new_f64_$R.log 2>&1 || exit $?
  AWQ_HIP_LIB=$PREV timeout -k 10 120 python scripts/generic_bench.py $GB > $OUT/prev_f64_$R.log 2>&1 || exit $?
done
timeout -k 10 120 python scripts/generic_bench.py $GD > $OUT/new_dequant.log 2>&1 || exit $?
AWQ_HIP_LIB=$PREV timeout -k 10 120 python scripts/generic_bench.py $GD > $OUT/prev_dequant.log 2>&1 || exit $?
timeout -k 10 120 python scripts/generic_bench.py $GB2 > $OUT/new_bf16_large.log 2>&1 || exit $?
AWQ_HIP_LIB=$PREV timeout -k 10 120 python scripts/generic_bench.py $GB2 > $OUT/prev_bf16_large.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_f64 -o f64 --output-format csv -- python scripts/generic_bench.py --shape 14336,4096 --dtypes f64 --group-sizes 128 > $OUT/prof_f64.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
echo done
