#!/bin/bash
# weight mean: Markstein quotient (product) vs the division (wm0): act GPU tests + block A/B
set -o pipefail
mkdir -p gpurun_out/r5m1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_act_search.py -m gpu > gpurun_out/r5m1/test.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 200 python scripts/act_search_bench.py --iters 10 --lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_wm0.so >> gpurun_out/r5m1/bench.log 2>&1 &&
  timeout -k 10 200 python scripts/act_search_bench.py --iters 10 >> gpurun_out/r5m1/bench.log 2>&1 || exit 1
done
