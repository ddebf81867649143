#!/bin/bash
# round 2: register-resident fp64 span (group sizes 64 / 128) — parity, then A/B against the
# strided span (AWQ_GEN_NOREG=1) and the round-start library, interleaved; rocprof stats of the
# fp64 launch and of the word-per-thread dequantize; dequantize and large-group A/B; the full
# GPU suite, smoke and the default bench line.
set -u
OUT=gpurun_out/r2an
mkdir -p $OUT
export TMPDIR=/tmp
PREV=awq-converter_amd/awq_quantizer/_lib/variants/prev/libawq_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_generic_span.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_span.log 2>&1 || exit $?
GB="--shape 14336,4096;4096,14336 --dtypes f64 --group-sizes 128,64,100"
for R in 1 2; do
  timeout -k 10 120 python scripts/generic_bench.py $GB > $OUT/reg_f64_$R.log 2>&1 || exit $?
  AWQ_GEN_NOREG=1 timeout -k 10 120 python scripts/generic_bench.py $GB > $OUT/noreg_f64_$R.log 2>&1 || exit $?
  AWQ_HIP_LIB=$PREV timeout -k 10 120 python scripts/generic_bench.py $GB > $OUT/prev_f64_$R.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o gen --output-format csv -- python scripts/generic_bench.py --shape 14336,4096 --dtypes f64,bf16 --group-sizes 128 --dequant > $OUT/prof.log 2>&1 || exit $?
GD="--shape 14336,4096;128256,4096 --dtypes bf16 --group-sizes 128,32 --dequant"
timeout -k 10 120 python scripts/generic_bench.py $GD > $OUT/new_dequant.log 2>&1 || exit $?
AWQ_HIP_LIB=$PREV timeout -k 10 120 python scripts/generic_bench.py $GD > $OUT/prev_dequant.log 2>&1 || exit $?
GB2="--shape 14336,4096 --dtypes bf16,f32 --group-sizes 1024,2048"
timeout -k 10 120 python scripts/generic_bench.py $GB2 > $OUT/new_large_groups.log 2>&1 || exit $?
AWQ_HIP_LIB=$PREV timeout -k 10 120 python scripts/generic_bench.py $GB2 > $OUT/prev_large_groups.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
echo done
