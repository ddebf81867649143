set -o pipefail
mkdir -p gpurun_out/r21
L=awq-converter_amd/awq_quantizer/_lib
V=$L/variants/libawq_hip_
AWQ_HIP_LIB=${V}p8.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fast or ragged or grid or golden or full" > gpurun_out/r21/pytest_p8.log 2>&1; rc=$?; tail -3 gpurun_out/r21/pytest_p8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/kbench.py --sets opt-125m,llama3-8b-mlp,k768,c1x64 --libs $L/libawq_hip.so,${V}p8.so,${V}p9.so,${V}p4.so,${V}p16.so,${V}p12.so --rounds 3 --iters 15 > gpurun_out/r21/kbench.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r21/kbench.log; exit $rc
