#!/bin/bash
# single-tensor launch loss: per-wave trace of one 128256x4096 launch vs the
# Llama-3-8B set, and per-launch times in idle / warm / paired clock states
set -o pipefail
OUT=gpurun_out/r6h
mkdir -p $OUT
timeout -k 10 300 python scripts/single_launch_bench.py > $OUT/single.log 2>&1 &&
timeout -k 10 200 python scripts/trace_waves.py --lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_trace.so --set lm-head-8b > $OUT/trace_lm_head.log 2>&1 &&
timeout -k 10 200 python scripts/trace_waves.py --lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_trace.so --set llama3-8b --reps 2 > $OUT/trace_llama3_8b.log 2>&1
echo rc=$?
timeout -k 10 300 python bench.py --mode search --workload llama3-8b --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_search.log 2>&1 &&
timeout -k 10 300 python bench.py --mode act --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_act.log 2>&1
echo rc=$?
