set -o pipefail
mkdir -p gpurun_out/r35
timeout -k 10 600 python -m pytest tests/test_gpu_f16_fast.py tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/r35/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r35/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/generic_bench.py --shape 14336,4096 > gpurun_out/r35/generic.log 2>&1 && grep '^{' gpurun_out/r35/generic.log || exit 1
timeout -k 10 600 python scripts/kbench.py --sets opt-125m,llama3-8b-mlp,c1x64 --dtype f16 --rounds 2 --iters 10 > gpurun_out/r35/kbench_f16.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r35/kbench_f16.log; exit $rc
