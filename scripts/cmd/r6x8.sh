#!/bin/bash
# fp16 group parameters without IEEE divisions (scale by RN(1/qr), rcp + Newton reciprocal checked
# by awq_selftest 2, Markstein zero-point quotient): full GPU suite first (every fp16 parity case),
# then kbench fp16 search A/B, act fp16 A/B, fp16 RTN single tensors, against the
# AWQ_F16_PARAMS_FAST=0 build
set -o pipefail
OUT=gpurun_out/r6x8
mkdir -p $OUT
P=awq-converter_amd/awq_quantizer/_lib
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python scripts/kbench.py --sets llama3-8b --search 10 --rounds 3 --iters 5 --dtype f16 --libs $P/libawq_hip.so,$P/ab/libawq_hip_f16prev.so > $OUT/kbench_f16_search.log 2>&1 &&
timeout -k 10 300 python scripts/kbench.py --sets llama3-8b --rounds 3 --iters 10 --dtype f16 --libs $P/libawq_hip.so,$P/ab/libawq_hip_f16prev.so > $OUT/kbench_f16_rtn.log 2>&1 || exit $?
for r in 1 2; do
  for L in $P/ab/libawq_hip_f16prev.so $P/libawq_hip.so; do
    timeout -k 10 200 python scripts/act_search_bench.py --dtype f16 --lib $L > $OUT/ab_$(basename $L .so)_f16_$r.log 2>&1 || exit $?
  done
done
echo rc=$?
