#!/bin/bash
# export v2 qweight kernel: GPU parity + A/B against the round-3 kernel
set -o pipefail
mkdir -p gpurun_out/r5e3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_autoawq_export.py -m gpu > gpurun_out/r5e3/test.log 2>&1 &&
timeout -k 10 120 python scripts/export_bench.py --lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_exv1.so > gpurun_out/r5e3/export_bench.log 2>&1 &&
timeout -k 10 120 python scripts/export_bench.py >> gpurun_out/r5e3/export_bench.log 2>&1
