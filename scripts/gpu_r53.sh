set -o pipefail
mkdir -p gpurun_out/r53
timeout -k 10 600 python -m pytest tests/test_gpu_f16_fast.py tests/test_gpu_parity.py tests/test_scale_search.py -m gpu -x -q > gpurun_out/r53/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r53/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/generic_bench.py --shape "14336,4096;4096,4096" --dtypes bf16,f16 --iters 50 > gpurun_out/r53/single.log 2>&1; rc=$?; grep '^{' gpurun_out/r53/single.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py --help > /dev/null 2>&1; timeout -k 10 400 python scripts/kbench.py --dtype f16 --rounds 3 --libs awq-converter_amd/awq_quantizer/_lib/libawq_hip.so,awq-converter_amd/awq_quantizer/_lib/variants/libawq_hip_f16mark.so > gpurun_out/r53/kbench_f16.log 2>&1; rc=$?; tail -12 gpurun_out/r53/kbench_f16.log; exit $rc
