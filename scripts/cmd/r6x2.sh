#!/bin/bash
# packed f32 pairs (v_pk_mul_f32 / v_pk_add_f32) in the bf16 search chain and the bf16 act tail
# (+ act launch bound of 3 waves) vs the previous commit: search / act GPU tests, bit check,
# kbench search A/B (bf16, fp16), act loss A/B (bf16, fp16)
set -o pipefail
OUT=gpurun_out/r6x2
mkdir -p $OUT
P=awq-converter_amd/awq_quantizer/_lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_scale_search.py tests/test_gpu_configs.py tests/test_act_search.py > $OUT/tests.log 2>&1 &&
timeout -k 10 120 python scripts/ab_search_check.py $P/libawq_hip.so > $OUT/check.log 2>&1 &&
timeout -k 10 300 python scripts/kbench.py --sets llama3-8b --search 10 --rounds 3 --iters 5 --libs $P/libawq_hip.so,$P/ab/libawq_hip_searchprev.so > $OUT/kbench_bf16.log 2>&1 &&
timeout -k 10 300 python scripts/kbench.py --sets llama3-8b --search 10 --rounds 3 --iters 5 --dtype f16 --libs $P/libawq_hip.so,$P/ab/libawq_hip_searchprev.so > $OUT/kbench_f16.log 2>&1 || exit $?
for r in 1 2; do
  for L in $P/ab/libawq_hip_actprev.so $P/libawq_hip.so; do
    for d in bf16 f16; do
      timeout -k 10 200 python scripts/act_search_bench.py --dtype $d --lib $L > $OUT/ab_$(basename $L .so)_${d}_$r.log 2>&1 || exit $?
    done
  done
done
echo rc=$?
