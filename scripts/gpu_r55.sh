set -o pipefail
mkdir -p gpurun_out/r55
L=awq-converter_amd/awq_quantizer/_lib
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_f16_fast.py tests/test_scale_search.py -m gpu -x -q > gpurun_out/r55/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r55/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/kbench.py --rounds 5 --libs $L/libawq_hip.so,$L/variants/libawq_hip_prev.so > gpurun_out/r55/kbench_bf16.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r55/kbench_bf16.log | tail -9; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/kbench.py --rounds 5 --dtype f16 --libs $L/libawq_hip.so,$L/variants/libawq_hip_prev.so > gpurun_out/r55/kbench_f16.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r55/kbench_f16.log | tail -9; exit $rc
