#!/bin/bash
# export: nontemporal threshold / nontemporal loads / grid order A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5e7
AB=awq-converter_amd/awq_quantizer/_lib/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_autoawq_export.py -m gpu > gpurun_out/r5e7/test.log 2>&1 &&
timeout -k 10 120 python scripts/export_bench.py --iters 50 > gpurun_out/r5e7/export_bench.log 2>&1 &&
for v in exnt0 exntld exntnf; do
  timeout -k 10 120 python scripts/export_bench.py --iters 50 --lib $AB/libawq_hip_$v.so >> gpurun_out/r5e7/export_bench.log 2>&1 || exit 1
done &&
timeout -k 10 120 python scripts/export_bench.py --iters 50 >> gpurun_out/r5e7/export_bench.log 2>&1
