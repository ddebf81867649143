#!/bin/bash
# export v2 with LDS group kernel: GPU parity + kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5e5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_autoawq_export.py -m gpu > gpurun_out/r5e5/test.log 2>&1 &&
timeout -k 10 120 python scripts/export_bench.py > gpurun_out/r5e5/export_bench.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e5/prof -o run -- python3 scripts/export_bench.py > gpurun_out/r5e5/prof.log 2>&1
