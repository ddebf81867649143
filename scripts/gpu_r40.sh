set -o pipefail
mkdir -p gpurun_out/r40
timeout -k 10 600 python -m pytest tests/test_scale_search.py tests/test_gpu_parity.py tests/test_gpu_f16_fast.py -m gpu -x -q > gpurun_out/r40/pytest.log 2>&1; rc=$?; tail -4 gpurun_out/r40/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16,f16 --search 10 --iters 5 > gpurun_out/r40/search.log 2>&1 && grep '^{' gpurun_out/r40/search.log
