#!/bin/bash
# round 2: extra bench lines on the final tree (fp16 / fp32 weights of the Llama-3-70B set,
# Llama-3-8B set) and HBM traffic of the packed dequantize and fp64 span kernels (separate
# FETCH_SIZE / WRITE_SIZE passes, kernel-trace only).
set -u
OUT=gpurun_out/r2as
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --dtype f16 --no-cpu-baseline > $OUT/bench_f16.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload llama3-8b --no-cpu-baseline > $OUT/bench_llama3-8b.log 2>&1 || exit $?
GB="--shape 14336,4096 --dtypes f64 --group-sizes 128 --dequant --iters 3"
timeout -s KILL 120 rocprofv3 --kernel-include-regex 'awq_dequant_words|awq_generic_span_reg' --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o gen -- python scripts/generic_bench.py $GB > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-include-regex 'awq_dequant_words|awq_generic_span_reg' --pmc WRITE_SIZE --output-format csv -d $OUT/write -o gen -- python scripts/generic_bench.py $GB > $OUT/write.log 2>&1 || exit $?
echo done
