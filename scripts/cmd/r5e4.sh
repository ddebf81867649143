#!/bin/bash
# export v2 with 16-B loads: GPU parity + A/B against 4-B loads + kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5e4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_autoawq_export.py -m gpu > gpurun_out/r5e4/test.log 2>&1 &&
timeout -k 10 120 python scripts/export_bench.py --lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_exld4.so > gpurun_out/r5e4/export_bench.log 2>&1 &&
timeout -k 10 120 python scripts/export_bench.py >> gpurun_out/r5e4/export_bench.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e4/prof -o run -- python3 scripts/export_bench.py > gpurun_out/r5e4/prof.log 2>&1
