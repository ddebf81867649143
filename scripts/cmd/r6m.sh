#!/bin/bash
# act loss kernel round-6 trims (NaN hoist, NaN-encoded reciprocal table, fp16 dq into v_fma_mix):
# the act-search GPU tests on the new default, then the A/B against the round-5 kernel (bf16, fp16)
set -o pipefail
OUT=gpurun_out/r6m
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_act_search.py > $OUT/tests.log 2>&1 &&
for r in 1 2; do
  for L in actr5 actnew; do
    for d in bf16 f16; do
      timeout -k 10 200 python scripts/act_search_bench.py --dtype $d --lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_$L.so > $OUT/ab_${L}_${d}_$r.log 2>&1 || exit $?
    done
  done
done
echo rc=$?
