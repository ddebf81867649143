#!/bin/bash
# act loss kernel: the reciprocal row read as (j, j + 8) pairs by ds_read2_b32 (no re-pairing movs) vs HEAD
# commit; act GPU tests; helpers
set -o pipefail
OUT=gpurun_out/r6x7
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_act_search.py tests/test_gpu_helpers.py > $OUT/tests.log 2>&1 &&
for r in 1 2; do
  for L in awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_actprev.so awq-converter_amd/awq_quantizer/_lib/libawq_hip.so; do
    for d in bf16 f16; do
      timeout -k 10 200 python scripts/act_search_bench.py --dtype $d --lib $L > $OUT/ab_$(basename $L .so)_${d}_$r.log 2>&1 || exit $?
    done
  done
done
echo rc=$?
