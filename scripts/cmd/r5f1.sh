#!/bin/bash
# quantize kernel: nt input loads (product) vs plain input loads (ld0), interleaved
set -o pipefail
mkdir -p gpurun_out/r5f1
timeout -k 10 400 python scripts/kbench.py --sets llama3-8b-mlp,llama3-8b,opt-125m --rounds 3 \
  --libs awq-converter_amd/awq_quantizer/_lib/libawq_hip.so,awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_ld0.so > gpurun_out/r5f1/kbench.log 2>&1
