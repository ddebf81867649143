#!/bin/bash
# act loss kernel: the w * s products as v_pk_mul_f32 pairs too (AWQ_ACT_PK_F32=2, built as
# ab/libawq_hip_actprev.so for this run; per-item spills outside the candidate loop) vs the
# committed kernel; two rounds, bf16 / fp16
set -o pipefail
OUT=gpurun_out/r6x4
mkdir -p $OUT
P=awq-converter_amd/awq_quantizer/_lib
for r in 1 2; do
  for L in $P/ab/libawq_hip_actprev.so $P/libawq_hip.so; do
    for d in bf16 f16; do
      timeout -k 10 200 python scripts/act_search_bench.py --dtype $d --lib $L > $OUT/ab_$(basename $L .so)_${d}_$r.log 2>&1 || exit $?
    done
  done
done
echo rc=$?
