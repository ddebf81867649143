set -o pipefail
mkdir -p gpurun_out/r39
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r39/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r39/pytest.log; exit $rc
