set -o pipefail
mkdir -p gpurun_out/r33
timeout -k 10 300 python scripts/generic_bench.py --shape 14336,4096 > gpurun_out/r33/generic.log 2>&1 && grep '^{' gpurun_out/r33/generic.log
timeout -k 10 300 python scripts/generic_bench.py --shape 4096,4096 --dtypes bf16,f16 --search 10 --iters 5 > gpurun_out/r33/search.log 2>&1 && grep '^{' gpurun_out/r33/search.log
