set -o pipefail
mkdir -p gpurun_out/r36
for f in packed reference; do
  timeout -k 10 600 python scripts/cli_bench.py --workload opt-125m --format $f > gpurun_out/r36/cli_$f.log 2>&1 || { tail -20 gpurun_out/r36/cli_$f.log; exit 1; }
  grep '^{' gpurun_out/r36/cli_$f.log
done
timeout -k 10 900 python scripts/cli_bench.py --workload opt-350m --format packed --repeat 1 > gpurun_out/r36/cli_350.log 2>&1 && grep '^{' gpurun_out/r36/cli_350.log
