#!/bin/bash
# dequantize_packed with plain qweight loads: dequant GPU tests + bench
set -o pipefail
mkdir -p gpurun_out/r5d2
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_generic_span.py tests/test_gpu_group_sizes.py tests/test_gpu_large.py tests/test_gpu_nan.py tests/test_gpu_padded_rows.py tests/test_gpu_parity.py -k "dequant or dq" > gpurun_out/r5d2/test.log 2>&1 &&
timeout -k 10 200 python scripts/generic_bench.py --shape "14336,4096;4096,14336;128256,4096" --dtypes bf16,f16 --group-sizes 128,100 --dequant --iters 20 > gpurun_out/r5d2/dq.log 2>&1
