set -o pipefail
mkdir -p gpurun_out/r37
timeout -k 10 600 python -m pytest tests/test_cli.py tests/test_scale_search.py -m gpu -x -q > gpurun_out/r37/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r37/pytest.log; [ $rc -eq 0 ] || exit $rc
for f in packed reference; do
  timeout -k 10 600 python scripts/cli_bench.py --workload opt-125m --format $f --repeat 3 > gpurun_out/r37/cli_$f.log 2>&1 || { tail -20 gpurun_out/r37/cli_$f.log; exit 1; }
  grep '^{' gpurun_out/r37/cli_$f.log
done
timeout -k 10 900 python scripts/cli_bench.py --workload opt-350m --format packed --repeat 2 > gpurun_out/r37/cli_350.log 2>&1 && grep '^{' gpurun_out/r37/cli_350.log
