#!/bin/bash
# export v2 with grid order + nontemporal A/B + kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5e6
timeout -k 10 120 python scripts/export_bench.py > gpurun_out/r5e6/export_bench.log 2>&1 &&
timeout -k 10 120 python scripts/export_bench.py --lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_exnf.so >> gpurun_out/r5e6/export_bench.log 2>&1 &&
timeout -k 10 120 python scripts/export_bench.py --lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_exnt.so >> gpurun_out/r5e6/export_bench.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e6/prof -o run -- python3 scripts/export_bench.py --lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_exnf.so > gpurun_out/r5e6/prof.log 2>&1
