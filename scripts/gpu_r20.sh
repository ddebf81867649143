set -o pipefail
mkdir -p gpurun_out/r20
L=awq-converter_amd/awq_quantizer/_lib
V=$L/variants/libawq_hip_
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/r20/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r20/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/kbench.py --sets opt-125m,llama3-8b-mlp,k768,c1x64 --libs $L/libawq_hip.so,${V}old.so,${V}s0.so,${V}olds0.so,${V}c4s0.so,${V}trivns.so,${V}trivs0.so --rounds 3 --iters 15 > gpurun_out/r20/kbench.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r20/kbench.log; exit $rc
