#!/bin/bash
# clip search: reduce-scatter + one special-scale ballot per candidate (per-load uniform branch, 80 / 96 VGPRs)
# vs the previous commit; search / config GPU tests, kbench A/B (bf16, fp16), bit check
set -o pipefail
OUT=gpurun_out/r6s
mkdir -p $OUT
P=awq-converter_amd/awq_quantizer/_lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_scale_search.py tests/test_gpu_configs.py > $OUT/tests.log 2>&1 &&
timeout -k 10 120 python scripts/ab_search_check.py $P/libawq_hip.so > $OUT/check.log 2>&1 &&
timeout -k 10 300 python scripts/kbench.py --sets llama3-8b --search 10 --rounds 3 --iters 5 --libs $P/libawq_hip.so,$P/ab/libawq_hip_searchprev.so > $OUT/kbench_bf16.log 2>&1 &&
timeout -k 10 300 python scripts/kbench.py --sets llama3-8b --search 10 --rounds 3 --iters 5 --dtype f16 --libs $P/libawq_hip.so,$P/ab/libawq_hip_searchprev.so > $OUT/kbench_f16.log 2>&1
echo rc=$?
