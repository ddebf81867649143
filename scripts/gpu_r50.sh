set -o pipefail
mkdir -p gpurun_out/r50
timeout -k 10 600 python -m pytest tests/test_act_search.py -m gpu -x -q > gpurun_out/r50/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r50/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/act_search_bench.py --tokens 512 --grid 20 > gpurun_out/r50/act_bench.log 2>&1; rc=$?; grep '^{' gpurun_out/r50/act_bench.log; exit $rc
