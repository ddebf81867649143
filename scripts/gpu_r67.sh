set -o pipefail
# direct pread-into-pinned loader: CLI GPU tests, then CLI end-to-end A/B (direct vs mmap+copy)
mkdir -p gpurun_out/r67
timeout -k 10 400 python -u -m pytest tests/test_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r67/pytest_cli.log 2>&1; rc=$?; tail -2 gpurun_out/r67/pytest_cli.log; [ $rc -eq 0 ] || exit $rc
W=/tmp/awq_cli_work
for WL in llama3-8b; do
  timeout -k 10 400 python scripts/cli_bench.py --workload $WL --shards 4 --repeat 4 --workdir $W.$WL > gpurun_out/r67/cli_$WL.log 2>&1; rc=$?; grep '^{' gpurun_out/r67/cli_$WL.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
  AWQ_CLI_MMAP_READ=1 timeout -k 10 400 python scripts/cli_bench.py --workload $WL --shards 4 --repeat 4 --workdir $W.$WL > gpurun_out/r67/cli_${WL}_mmap.log 2>&1; rc=$?; grep '^{' gpurun_out/r67/cli_${WL}_mmap.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
  rm -rf $W.$WL
done
