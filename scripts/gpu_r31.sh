set -o pipefail
mkdir -p gpurun_out/r31
L=awq-converter_amd/awq_quantizer/_lib
V=$L/variants/libawq_hip_
AWQ_HIP_LIB=${V}w8ws.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fast or ragged or grid or golden or full or special" > gpurun_out/r31/pytest_w8ws.log 2>&1; rc=$?; tail -2 gpurun_out/r31/pytest_w8ws.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scripts/kbench.py --sets opt-125m,llama3-8b-mlp,k768,c1x64,c1 --libs $L/libawq_hip.so,${V}ws.so,${V}w8.so,${V}w16.so,${V}w8ws.so,${V}trivws.so --rounds 3 --iters 10 > gpurun_out/r31/kbench.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r31/kbench.log; exit $rc
