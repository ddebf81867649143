set -o pipefail
mkdir -p gpurun_out/r41
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r41/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r41/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r41/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r41/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r41/bench.json 2> gpurun_out/r41/bench.err; rc=$?; cat gpurun_out/r41/bench.json; exit $rc
