set -o pipefail
# group sizes 32/64/256 on the streaming kernel: parity first, then the in-process A/B of the
# gs-128 kernel (this build vs the previous commit's) and the new group sizes' throughput
mkdir -p gpurun_out/r57
L=awq-converter_amd/awq_quantizer/_lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_group_sizes.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r57/pytest_gs.log 2>&1; rc=$?; tail -3 gpurun_out/r57/pytest_gs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r57/pytest_all.log 2>&1; rc=$?; tail -3 gpurun_out/r57/pytest_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/kbench.py --rounds 5 --libs $L/libawq_hip.so,$L/variants/libawq_hip_prev.so > gpurun_out/r57/kbench_bf16.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r57/kbench_bf16.log | tail -9; [ $rc -eq 0 ] || exit $rc
for GS in 32 64 256; do
timeout -k 10 300 python scripts/kbench.py --rounds 3 --group-size $GS > gpurun_out/r57/kbench_gs$GS.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r57/kbench_gs$GS.log | tail -5; [ $rc -eq 0 ] || exit $rc
done
