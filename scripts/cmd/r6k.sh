#!/bin/bash
# clip search: x - dq as v_fma_mix_f32 on the fp16 product (AWQ_SEARCH_FMA_MIX=1) vs the round-5 chain;
# the search's GPU tests on the new default, then the A/B on the Llama-3-8B set (bf16, fp16)
set -o pipefail
OUT=gpurun_out/r6k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_scale_search.py tests/test_gpu_configs.py > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python scripts/kbench.py --sets llama3-8b --search 10 --rounds 3 --iters 5 --libs awq-converter_amd/awq_quantizer/_lib/libawq_hip.so,awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_searchr5.so > $OUT/kbench_bf16.log 2>&1 &&
timeout -k 10 300 python scripts/kbench.py --sets llama3-8b --search 10 --rounds 3 --iters 5 --dtype f16 --libs awq-converter_amd/awq_quantizer/_lib/libawq_hip.so,awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_searchr5.so > $OUT/kbench_f16.log 2>&1
echo rc=$?
