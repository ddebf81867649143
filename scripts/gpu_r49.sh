set -o pipefail
mkdir -p gpurun_out/r49
timeout -k 10 600 python -m pytest tests/test_cli.py tests/test_act_search.py -m gpu -x -q > gpurun_out/r49/pytest.log 2>&1; rc=$?; tail -30 gpurun_out/r49/pytest.log; exit $rc
