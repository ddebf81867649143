#!/bin/bash
# dequantize_packed: nt qweight loads + nt stores (product) vs plain loads (dqld) vs plain stores (dqst)
set -o pipefail
mkdir -p gpurun_out/r5d1
AB=awq-converter_amd/awq_quantizer/_lib/ab
for L in "" $AB/libawq_hip_dqld.so $AB/libawq_hip_dqst.so "" $AB/libawq_hip_dqld.so $AB/libawq_hip_dqst.so; do
  timeout -k 10 120 python scripts/generic_bench.py --shape "14336,4096;4096,14336;128256,4096" --dtypes bf16 --group-sizes 128 --dequant --iters 20 ${L:+--lib $L} >> gpurun_out/r5d1/dq.log 2>&1 || exit 1
done
