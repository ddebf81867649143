set -o pipefail
# overlapped chunk writer: CLI GPU tests, then CLI end-to-end A/B (serial save vs overlapped)
mkdir -p gpurun_out/r63
timeout -k 10 400 python -u -m pytest tests/test_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r63/pytest_cli.log 2>&1; rc=$?; tail -2 gpurun_out/r63/pytest_cli.log; [ $rc -eq 0 ] || exit $rc
W=/tmp/awq_cli_work
for WL in opt-350m llama3-8b; do
  timeout -k 10 400 python scripts/cli_bench.py --workload $WL --shards 4 --repeat 3 --workdir $W.$WL > gpurun_out/r63/cli_$WL.log 2>&1; rc=$?; grep '^{' gpurun_out/r63/cli_$WL.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
  AWQ_CLI_SERIAL_SAVE=1 timeout -k 10 400 python scripts/cli_bench.py --workload $WL --shards 4 --repeat 3 --workdir $W.$WL > gpurun_out/r63/cli_${WL}_serial.log 2>&1; rc=$?; grep '^{' gpurun_out/r63/cli_${WL}_serial.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
  rm -rf $W.$WL
done
