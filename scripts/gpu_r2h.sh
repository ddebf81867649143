#!/bin/bash
# round 2: trivial-compute A/B at one wave per workgroup, then the default bench line and
# its rocprofv3 evidence (kernel trace + FETCH_SIZE / WRITE_SIZE passes) for llama3-70b.
set -u
OUT=gpurun_out/r2h
mkdir -p $OUT
export TMPDIR=/tmp
V=awq-converter_amd/awq_quantizer/_lib/variants
L=awq-converter_amd/awq_quantizer/_lib/libawq_hip.so
timeout -k 10 300 python scripts/kbench.py --sets llama3-8b,opt-125m --libs $L,$V/libawq_hip_triv1.so --rounds 3 --iters 20 > $OUT/kbench_triv1.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || exit $?
COMMIT=${COMMIT:-unknown} STEP_TIMEOUT=300 bash scripts/profile_round.sh r2h/prof || exit $?
echo done
