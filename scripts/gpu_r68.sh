set -o pipefail
# padded rows on the streaming kernel: parity, full suite, gs-128 A/B vs the previous build, a Falcon-like set
mkdir -p gpurun_out/r68
L=awq-converter_amd/awq_quantizer/_lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_padded_rows.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r68/pytest_pad.log 2>&1; rc=$?; tail -3 gpurun_out/r68/pytest_pad.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r68/pytest_all.log 2>&1; rc=$?; tail -2 gpurun_out/r68/pytest_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/kbench.py --rounds 5 --libs $L/libawq_hip.so,$L/variants/libawq_hip_prev.so > gpurun_out/r68/kbench_bf16.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r68/kbench_bf16.log | tail -9; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py --rounds 3 --sets falcon7b-mlp > gpurun_out/r68/kbench_falcon.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r68/kbench_falcon.log | tail -3; exit $rc
