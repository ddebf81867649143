#!/bin/bash
# dequantize_packed on the Llama-3-8B lm_head: store-ceiling probe (2 GB footprint, past the MALL),
# the kernel timed, and its FETCH_SIZE / WRITE_SIZE passes (each its own rocprofv3 run)
set -o pipefail
OUT=gpurun_out/r6e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 ./scripts/dq_probe > $OUT/dq_probe.log 2>&1 &&
timeout -k 10 200 python scripts/dq_pmc_driver.py --iters 20 > $OUT/dq_time.log 2>&1 &&
timeout -k 10 200 python scripts/generic_bench.py --shape "128256,4096" --dtypes bf16 --group-sizes 128 --dequant --iters 20 > $OUT/dq_bench.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex awq_dequant_batch_kernel --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o p -- python scripts/dq_pmc_driver.py > $OUT/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex awq_dequant_batch_kernel --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o p -- python scripts/dq_pmc_driver.py > $OUT/pmc_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex awq_dequant_batch_kernel --output-format csv -d $OUT/trace -o p -- python scripts/dq_pmc_driver.py > $OUT/trace.log 2>&1
echo rc=$?
