set -o pipefail
mkdir -p gpurun_out/r22
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r22/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r22/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r22/bench.json 2> gpurun_out/r22/bench.err; rc=$?; cat gpurun_out/r22/bench.json; exit $rc
