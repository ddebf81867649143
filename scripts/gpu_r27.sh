set -o pipefail
mkdir -p gpurun_out/r27
L=awq-converter_amd/awq_quantizer/_lib
V=$L/variants/libawq_hip_
timeout -k 10 900 python scripts/kbench.py --sets opt-125m,llama3-8b-mlp,k768,c1x64,c1 --libs $L/libawq_hip.so,${V}pf0.so,${V}pf1.so --blocks 0,t1,t2,t4 --rounds 3 --iters 10 > gpurun_out/r27/kbench.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r27/kbench.log; exit $rc
