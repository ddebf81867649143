#!/bin/bash
# export kernels (final round-5 form): GPU parity + bench + kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5e8
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_autoawq_export.py -m gpu > gpurun_out/r5e8/test.log 2>&1 &&
timeout -k 10 120 python scripts/export_bench.py --iters 50 > gpurun_out/r5e8/export_bench.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e8/prof -o run -- python3 scripts/export_bench.py > gpurun_out/r5e8/prof.log 2>&1
