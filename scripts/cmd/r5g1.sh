#!/bin/bash
# row-segment kernel: nt input loads (product) vs plain loads (rgld), on shapes past the MALL and a mid one
set -o pipefail
mkdir -p gpurun_out/r5g1
AB=awq-converter_amd/awq_quantizer/_lib/ab
for L in "" $AB/libawq_hip_rgld.so "" $AB/libawq_hip_rgld.so; do
  timeout -k 10 150 python scripts/generic_bench.py --shape "128256,4096;57344,8192;14336,4096" --dtypes bf16,f16 --group-sizes 100 --iters 20 ${L:+--lib $L} >> gpurun_out/r5g1/rg.log 2>&1 || exit 1
done
