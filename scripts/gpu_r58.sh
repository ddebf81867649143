set -o pipefail
# fp32 on the streaming kernel: parity, full GPU suite, then throughput (fp32 sets; bf16 A/B)
mkdir -p gpurun_out/r58
L=awq-converter_amd/awq_quantizer/_lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32_fast.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r58/pytest_f32.log 2>&1; rc=$?; tail -3 gpurun_out/r58/pytest_f32.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r58/pytest_all.log 2>&1; rc=$?; tail -3 gpurun_out/r58/pytest_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py --rounds 3 --dtype f32 > gpurun_out/r58/kbench_f32.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r58/kbench_f32.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/kbench.py --rounds 5 --libs $L/libawq_hip.so,$L/variants/libawq_hip_prev.so > gpurun_out/r58/kbench_bf16.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r58/kbench_bf16.log | tail -9; exit $rc
