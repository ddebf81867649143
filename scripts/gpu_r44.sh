set -o pipefail
mkdir -p gpurun_out/r44
timeout -k 10 1000 python scripts/cli_bench.py --workload llama3-8b --format packed --shards 4 --repeat 2 > gpurun_out/r44/cli_8b.log 2>&1; rc=$?; grep '^{' gpurun_out/r44/cli_8b.log; tail -3 gpurun_out/r44/cli_8b.log; exit $rc
