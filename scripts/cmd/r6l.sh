#!/bin/bash
# which search change breaks fp16: product (fma_mix, s broadcast as before), slate (+ late s), searchr5 (no fma_mix)
OUT=gpurun_out/r6l
mkdir -p $OUT
for L in awq-converter_amd/awq_quantizer/_lib/libawq_hip.so awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_slate.so awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_searchr5.so; do
  timeout -k 10 120 python scripts/ab_search_check.py $L >> $OUT/check.log 2>&1; rc=$?
  echo "$L rc=$rc" >> $OUT/check.log
  case $rc in 0|1) ;; *) exit $rc;; esac
done
