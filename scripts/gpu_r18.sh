set -o pipefail
mkdir -p gpurun_out/r19
L=awq-converter_amd/awq_quantizer/_lib
V=$L/variants/libawq_hip_
timeout -k 10 600 python scripts/kbench.py --sets opt-125m,llama3-8b-mlp,k768,c1x64 --libs $L/libawq_hip.so,${V}s0.so,${V}x.so,${V}xs0.so,${V}xc4s0.so,${V}c4s0.so,${V}trivxs0.so,${V}trivns.so --rounds 3 --iters 15 > gpurun_out/r19/kbench.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r19/kbench.log; exit $rc
